"""sahajBERT tokenizer: training and the transformers wrapper (D12).

Reference behaviour: ``sahajbert/tokenizer/tokenizer_model.py:9-87`` (SentencePiece-style Unigram
with Bengali normalisation), ``tokenizer_training_custom.py:6-31`` (vocabulary 31,995 + 5 special
tokens trained on OSCAR-bn) and the manual post-training edits of ``tokenizer/README.md:12-19``
(``[MASK]`` gets ``lstrip`` so it swallows the preceding space like a word, ``unk_id`` = 1), which
are applied programmatically here; ``tokenization_albert_bengali_fast.py:19-103`` (fast tokenizer
with the ALBERT special tokens, max length 512).

Pipeline:
  normalizer      NMT cleanup, NFKC, collapse runs of spaces, Bengali punctuation unification
                  (U+09E4/U+09E5 -> danda/double danda U+0964/U+0965, '|' and U+09F7 -> danda,
                  ':' after a Bengali letter -> visarga U+0983), lowercase
  pre-tokenizer   Metaspace('▁', prefix space), every digit its own piece, punctuation split
  post-processor  [CLS] A [SEP] (pair: [CLS] A [SEP] B [SEP], B with token type 1)

No corpus download is possible here: ``--input`` points at local text (files or directories of .txt,
one document per blank-line-separated block, as in ``data/sop_dataset.py``).
"""
from __future__ import annotations

import argparse
import json
import os
from typing import Iterable, List, Optional

SPECIAL_TOKENS = ("<pad>", "<unk>", "[CLS]", "[SEP]", "[MASK]")  # ids 0..4
DEFAULT_VOCAB = 31_995 + len(SPECIAL_TOKENS)


def bengali_pipeline(model=None):
    """A ``tokenizers.Tokenizer`` with the sahajBERT normalizer / pre-tokenizer / decoder / template
    around ``model`` (an untrained Unigram by default)."""
    from tokenizers import Regex, Tokenizer, decoders, normalizers, pre_tokenizers
    from tokenizers.models import Unigram
    from tokenizers.processors import TemplateProcessing

    tok = Tokenizer(model if model is not None else Unigram())
    bengali_punct = [("৤", "।"), ("৥", "॥"), ("|", "।"), ("৷", "।")]
    tok.normalizer = normalizers.Sequence(
        [normalizers.Nmt(), normalizers.NFKC(), normalizers.Replace(Regex(" {2,}"), " ")]
        + [normalizers.Replace(a, b) for a, b in bengali_punct]
        + [normalizers.Replace(Regex(r"(?<=[ঀ-৿]):"), "ঃ"), normalizers.Lowercase()])
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="always"),
        pre_tokenizers.Digits(individual_digits=True),
        pre_tokenizers.Punctuation()])
    tok.decoder = decoders.Metaspace(replacement="▁", prepend_scheme="always")
    cls, sep = SPECIAL_TOKENS.index("[CLS]"), SPECIAL_TOKENS.index("[SEP]")
    tok.post_processor = TemplateProcessing(single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B:1 [SEP]:1",
                                            special_tokens=[("[CLS]", cls), ("[SEP]", sep)])
    return tok


def _finalize(tok):
    """The reference README's manual edits: ``[MASK]`` lstrip and ``unk_id`` = id of ``<unk>``."""
    from tokenizers import Tokenizer

    spec = json.loads(tok.to_str())
    for t in spec.get("added_tokens", []):
        if t["content"] == "[MASK]":
            t["lstrip"] = True
    if spec["model"].get("type") == "Unigram":
        spec["model"]["unk_id"] = SPECIAL_TOKENS.index("<unk>")
    return Tokenizer.from_str(json.dumps(spec))


def train_tokenizer(texts: Iterable[str], vocab_size: int = DEFAULT_VOCAB, show_progress: bool = False):
    """Train the Unigram model on ``texts`` (strings or batches of strings) and finalize it."""
    from tokenizers import trainers

    tok = bengali_pipeline()
    trainer = trainers.UnigramTrainer(vocab_size=vocab_size, special_tokens=list(SPECIAL_TOKENS),
                                      unk_token="<unk>", show_progress=show_progress)
    tok.train_from_iterator(texts, trainer=trainer)
    return _finalize(tok)


def AlbertBengaliTokenizerFast(tokenizer_file: Optional[str] = None, tokenizer_object=None, **kwargs):
    """``PreTrainedTokenizerFast`` with the sahajBERT special tokens (reference class of the same name):
    bos/cls ``[CLS]``, eos/sep ``[SEP]``, unk ``<unk>``, pad ``<pad>``, mask ``[MASK]``, max length 512."""
    from transformers import PreTrainedTokenizerFast

    defaults = dict(bos_token="[CLS]", eos_token="[SEP]", unk_token="<unk>", sep_token="[SEP]", pad_token="<pad>",
                    cls_token="[CLS]", mask_token="[MASK]", padding_side="right", model_max_length=512,
                    model_input_names=["input_ids", "token_type_ids", "attention_mask"])  # ALBERT's inputs
    defaults.update(kwargs)
    return PreTrainedTokenizerFast(tokenizer_file=tokenizer_file, tokenizer_object=tokenizer_object, **defaults)


def save_tokenizer(tok, output_dir: str):
    """Write a directory loadable by ``AutoTokenizer.from_pretrained`` (tokenizer.json +
    special_tokens_map.json + tokenizer_config.json), e.g. for ``run_trainer --tokenizer_path``."""
    AlbertBengaliTokenizerFast(tokenizer_object=tok).save_pretrained(output_dir)
    return output_dir


def _texts(paths: List[str], batch: int = 100):
    from .sop_dataset import read_documents

    buf = []
    for p in paths:
        for doc in read_documents(p):
            buf.append(doc)
            if len(buf) == batch:
                yield buf
                buf = []
    if buf:
        yield buf


def main(argv=None):
    ap = argparse.ArgumentParser(description="train the sahajBERT Unigram tokenizer on local text")
    ap.add_argument("--input", nargs="+", required=True, help="text files or directories of .txt files")
    ap.add_argument("--output_dir", required=True)
    ap.add_argument("--vocab_size", type=int, default=DEFAULT_VOCAB)
    a = ap.parse_args(argv)
    tok = train_tokenizer(_texts(a.input), vocab_size=a.vocab_size, show_progress=True)
    os.makedirs(a.output_dir, exist_ok=True)
    save_tokenizer(tok, a.output_dir)
    print(json.dumps({"output_dir": a.output_dir, "vocab_size": tok.get_vocab_size()}))


if __name__ == "__main__":
    main()
