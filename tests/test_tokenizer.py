"""sahajBERT tokenizer: Bengali normalisation, the Unigram training recipe with the
reference README's post-training edits, the transformers wrapper, and tokenization parity with the
reference's shipped ``sahajbert/tokenizer/data/tokenizer.json`` (read as JSON; skipped when the
reference tree is absent, e.g. on the GPU box)."""
import json
import os
import random
import subprocess
import sys

import pytest

from dedloc_amd.data.tokenizer import (SPECIAL_TOKENS, AlbertBengaliTokenizerFast, bengali_pipeline, save_tokenizer,
                                       train_tokenizer)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_TOKENIZER = "/root/reference/sahajbert/tokenizer/data/tokenizer.json"
LETTERS = "অআইঈউএওকখগঘচছজঝটঠডঢতথদধনপফবভমযরলশষসহড়য়"
SIGNS = "ািীুূেৈোৌং"


def _corpus(n_docs=120, seed=0):
    rng = random.Random(seed)
    words = ["".join(rng.choice(LETTERS) + (rng.choice(SIGNS) if rng.random() < 0.6 else "")
                     for _ in range(rng.randint(1, 4))) for _ in range(300)]
    docs = []
    for _ in range(n_docs):
        sents = [" ".join(rng.choice(words) for _ in range(rng.randint(3, 10))) + rng.choice(["।", "?", "!"])
                 for _ in range(rng.randint(1, 6))]
        docs.append(" ".join(sents))
    return docs


def test_bengali_normalizer():
    norm = bengali_pipeline().normalizer
    assert norm.normalize_str("ক৤ খ৥ গ| ঘ৷") == "ক। খ॥ গ। ঘ।"
    assert norm.normalize_str("নমস্কার:  Hello   World") == "নমস্কারঃ hello world"
    assert norm.normalize_str("a: b") == "a: b"  # visarga only after a Bengali letter
    pre = bengali_pipeline().pre_tokenizer.pre_tokenize_str("দাম ১২৩, ঠিক!")
    assert [p for p, _ in pre] == ["▁দাম", "▁", "১", "২", "৩", ",", "▁ঠিক", "!"]


def test_train_and_wrap(tmp_path):
    tok = train_tokenizer(_corpus(), vocab_size=300)
    assert 100 < tok.get_vocab_size() <= 300
    assert [tok.token_to_id(t) for t in SPECIAL_TOKENS] == [0, 1, 2, 3, 4]
    spec = json.loads(tok.to_str())
    assert spec["model"]["unk_id"] == 1
    assert [t["lstrip"] for t in spec["added_tokens"] if t["content"] == "[MASK]"] == [True]
    save_tokenizer(tok, str(tmp_path / "tok"))
    from transformers import AutoTokenizer

    hf = AutoTokenizer.from_pretrained(str(tmp_path / "tok"))
    assert (hf.pad_token_id, hf.unk_token_id, hf.cls_token_id, hf.sep_token_id, hf.mask_token_id) == (0, 1, 2, 3, 4)
    assert hf.model_max_length == 512
    enc = hf("আমি [MASK] খাই।", "তুমি কি খাও?")
    ids = enc["input_ids"]
    assert ids[0] == 2 and ids[-1] == 3 and ids.count(3) == 2 and 4 in ids
    assert ids[ids.index(4) - 1] != hf.convert_tokens_to_ids("▁")  # lstrip: the space goes with [MASK]
    first_sep = ids.index(3)
    assert set(enc["token_type_ids"][:first_sep + 1]) == {0} and set(enc["token_type_ids"][first_sep + 1:]) == {1}


@pytest.mark.skipif(not os.path.exists(REF_TOKENIZER), reason="reference tokenizer artifact not present")
def test_pipeline_parity_with_reference_artifact():
    """Our normalizer / pre-tokenizer / template around the reference's trained Unigram model encode
    exactly like the reference's tokenizer.json."""
    from tokenizers import Tokenizer

    ref = Tokenizer.from_file(REF_TOKENIZER)
    ours = bengali_pipeline(model=Tokenizer.from_file(REF_TOKENIZER).model)
    ours.add_special_tokens(list(SPECIAL_TOKENS))
    ours = Tokenizer.from_str(ours.to_str())
    assert ours.get_vocab_size() == ref.get_vocab_size() == 32000
    texts = ["আমি বাংলায় গান গাই৤ ১২৩ Hello, World!", "সে বলল: 'চলো'  |  দাম ৫০০ টাকা৷",
             "ঢাকা বাংলাদেশের রাজধানী। জনসংখ্যা প্রায় ২,০০,০০,০০০।", "MiXeD   case  টেক্সট ৥ end"]
    for a, b in zip(texts, texts[1:] + texts[:1]):
        assert ours.encode(a).ids == ref.encode(a).ids
        assert ours.encode(a, b).ids == ref.encode(a, b).ids
        assert ours.encode(a, b).type_ids == ref.encode(a, b).type_ids
    wrapped = AlbertBengaliTokenizerFast(tokenizer_file=REF_TOKENIZER)
    assert len(wrapped) == 32000 and wrapped.mask_token_id == 4 and wrapped.unk_token_id == 1


@pytest.mark.timeout(240)
def test_cli_trains_a_tokenizer_for_streaming(tmp_path):
    """CLI -> tokenizer directory -> the sahajBERT streaming SOP stream (D11) tokenizes with it."""
    (tmp_path / "bn.txt").write_text("\n\n".join(_corpus(200, seed=1)) + "\n", encoding="utf-8")
    r = subprocess.run([sys.executable, "-m", "dedloc_amd.data.tokenizer", "--input", str(tmp_path / "bn.txt"),
                        "--output_dir", str(tmp_path / "tok"), "--vocab_size", "400"], cwd=ROOT,
                       capture_output=True, text=True, timeout=200, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    from transformers import AutoTokenizer

    from dedloc_amd.data.sop_dataset import StreamingSOPStream

    hf = AutoTokenizer.from_pretrained(str(tmp_path / "tok"))
    s = StreamingSOPStream([(str(tmp_path / "bn.txt"), 1.0)], hf, batch_size=4, seed=0, max_seq_length=64,
                           shuffle_buffer=32)
    b = s.next_batch()
    assert b["input_ids"].shape[0] == 4 and (b["input_ids"][:, 0] == hf.cls_token_id).all()
    assert int(b["input_ids"].max()) < len(hf)
