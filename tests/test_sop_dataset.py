"""Real-text SOP data path (reference albert/tokenize_wikitext103.py): instance
construction semantics, the on-disk dataset + tokenizer metadata, HF-collator-style MLM masking of
the device batches, and a run_trainer peer training on the built dataset (BASELINE config 1 shape).

No network: the tokenizer is a WordPiece model trained here with `tokenizers` on the test corpus
(parity with the reference's albert-large-v2 sentencepiece vocabulary is unpinned; only the
instance / collator semantics are checked)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from dedloc_amd.data.sop_dataset import (DiskSOPStream, SOPInstanceBuilder, build_dataset, read_documents,
                                         split_sentences)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORD = ["zero", "one", "two", "three", "four", "five", "six", "seven", "eight", "nine", "ten", "eleven",
       "twelve", "thirteen", "fourteen", "fifteen", "sixteen", "seventeen", "eighteen", "nineteen"]
WORDS = ["river", "stone", "light", "green", "house", "music", "paper", "cloud", "train", "garden", "window",
         "ocean", "forest", "winter", "summer", "bridge", "market", "silver", "yellow", "people"]


def _corpus(n_docs=40, seed=0):
    import random

    rng = random.Random(seed)
    docs = []
    for _ in range(n_docs):
        n = rng.randint(1, 12)
        sents = [" ".join([ORD[i]] + [rng.choice(WORDS) for _ in range(rng.randint(3, 12))]) + "."
                 for i in range(n)]
        docs.append(" ".join(sents))
    return docs


@pytest.fixture(scope="module")
def tokenizer(tmp_path_factory):
    from tokenizers import Tokenizer, models, pre_tokenizers, processors, trainers
    from transformers import PreTrainedTokenizerFast

    tok = Tokenizer(models.WordPiece(unk_token="[UNK]"))
    tok.pre_tokenizer = pre_tokenizers.Whitespace()
    trainer = trainers.WordPieceTrainer(vocab_size=200, special_tokens=["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"])
    tok.train_from_iterator(_corpus(200, seed=1), trainer)
    cls, sep = tok.token_to_id("[CLS]"), tok.token_to_id("[SEP]")
    tok.post_processor = processors.TemplateProcessing(single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B:1 [SEP]:1",
                                                       special_tokens=[("[CLS]", cls), ("[SEP]", sep)])
    fast = PreTrainedTokenizerFast(tokenizer_object=tok, unk_token="[UNK]", pad_token="[PAD]", cls_token="[CLS]",
                                   sep_token="[SEP]", mask_token="[MASK]")
    d = tmp_path_factory.mktemp("tok")
    fast.save_pretrained(str(d))
    return fast, str(d)


def test_split_sentences():
    assert split_sentences("One two. Three four!  Five? six") == ["One two.", "Three four!", "Five?", "six"]
    assert split_sentences("আমি ভাত খাই। তুমি কি খাও?") == ["আমি ভাত খাই।", "তুমি কি খাও?"]


def test_instances_follow_reference_semantics(tokenizer):
    tok, _ = tokenizer
    b = SOPInstanceBuilder(tok, max_seq_length=48, seed=3)
    n_single = 0
    labels = []
    for doc in _corpus(60):
        insts = b.from_document(doc)
        if len(split_sentences(doc)) == 1:
            assert insts == []  # a one-sentence document yields no instance
            n_single += 1
        for inst in insts:
            ids = inst["input_ids"]
            assert len(ids) <= 48 and ids[0] == tok.cls_token_id and ids[-1] == tok.sep_token_id
            seps = [i for i, t in enumerate(ids) if t == tok.sep_token_id]
            assert len(seps) == 2
            assert inst["token_type_ids"] == [0] * (seps[0] + 1) + [1] * (len(ids) - seps[0] - 1)
            assert inst["special_tokens_mask"] == [int(t in (tok.cls_token_id, tok.sep_token_id)) for t in ids]
            # segment order: the first sentence ordinal of A vs B decides the label
            a_first = tok.convert_ids_to_tokens(ids[1])
            b_first = tok.convert_ids_to_tokens(ids[seps[0] + 1])
            if a_first in ORD and b_first in ORD:
                assert inst["sentence_order_label"] == int(ORD.index(a_first) > ORD.index(b_first))
            labels.append(inst["sentence_order_label"])
    assert n_single > 0 and 0.3 < sum(labels) / len(labels) < 0.7


def test_dataset_build_and_masked_batches(tokenizer, tmp_path):
    tok, _ = tokenizer
    corpus = tmp_path / "corpus.txt"
    corpus.write_text("\n\n".join(_corpus(80)) + "\n")
    docs = list(read_documents(str(corpus)))
    assert len(docs) == 80
    ds = build_dataset(docs, tok, str(tmp_path / "ds"), max_seq_length=64, seed=0)
    meta = json.load(open(tmp_path / "ds" / "sop_meta.json"))
    assert meta["mask"] == tok.mask_token_id and meta["vocab_size"] == len(tok) and meta["num_instances"] == len(ds)
    s = DiskSOPStream(str(tmp_path / "ds"), batch_size=8, seed=5)
    picked = masked = kept = total = 0
    for _ in range(40):
        b = s.next_batch()
        B, L = b["input_ids"].shape
        assert B == 8 and L <= 64 and b["sentence_order_label"].shape == (8,)
        real = b["attention_mask"].bool()
        lab = b["labels"]
        sel = lab != -100
        assert not (sel & ~real).any()  # never a padding position
        assert not (sel & ((lab == tok.cls_token_id) | (lab == tok.sep_token_id))).any()  # never a special token
        picked += int(sel.sum())
        total += int(real.sum()) - 3 * B
        masked += int((b["input_ids"][sel] == tok.mask_token_id).sum())
        kept += int((b["input_ids"][sel] == lab[sel]).sum())
    assert 0.12 < picked / total < 0.18
    assert 0.72 < masked / picked < 0.88 and 0.05 < kept / picked < 0.16


@pytest.mark.timeout(300)
def test_run_trainer_on_tokenized_dataset(tokenizer, tmp_path):
    """run_trainer with --dataset_path pointing at a built dataset trains on it (embeddings resized
    to the tokenizer like the reference's get_model)."""
    from dedloc_amd.dht import DHT
    from dedloc_amd.models.albert import AlbertConfig

    tok, tok_dir = tokenizer
    (tmp_path / "c.txt").write_text("\n\n".join(_corpus(60)) + "\n")
    r = subprocess.run([sys.executable, "-m", "dedloc_amd.data.sop_dataset", "--input", str(tmp_path / "c.txt"),
                        "--tokenizer", tok_dir, "--output_dir", str(tmp_path / "ds"), "--max_seq_length", "64"],
                       cwd=ROOT, capture_output=True, text=True, timeout=120, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    cfgdir = tmp_path / "cfg"
    AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64).save_pretrained(str(cfgdir))
    root = DHT(listen_on="127.0.0.1:*")
    try:
        metrics = tmp_path / "m.jsonl"
        cmd = [sys.executable, "-m", "dedloc_amd.cli.run_trainer", "--experiment_prefix", "sop",
               "--initial_peers", root.endpoint, "--device", "cpu", "--config_path", str(cfgdir),
               "--dataset_path", str(tmp_path / "ds"), "--per_device_train_batch_size", "2",
               "--gradient_accumulation_steps", "1", "--target_batch_size", "4", "--stop_after_global_steps", "2",
               "--save_steps", "0", "--output_dir", str(tmp_path / "out"), "--min_refresh_period", "0.05",
               "--default_refresh_period", "0.1", "--dht_listen_on", "127.0.0.1:*", "--listen_on", "127.0.0.1:*",
               "--metrics_file", str(metrics)]
        env = dict(os.environ, PYTHONPATH=ROOT)
        env.pop("RANK", None)
        env.pop("WORLD_SIZE", None)
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        assert "training on the tokenized dataset" in r.stderr
        recs = [json.loads(x) for x in metrics.read_text().splitlines()]
        assert max(rec["step"] for rec in recs) >= 2 and all(torch.isfinite(torch.tensor(rec["loss"])) for rec in recs)
    finally:
        root.shutdown()


def test_parse_sources():
    from dedloc_amd.data.sop_dataset import parse_sources

    assert parse_sources("a/wiki:0.23, b/oscar:0.77") == [("a/wiki", 0.23), ("b/oscar", 0.77)]
    assert parse_sources("corpus.txt") == [("corpus.txt", 1.0)]
    assert parse_sources("c:/x/y.txt:2,") == [("c:/x/y.txt", 2.0)]


def test_streaming_mixture_and_endless(tokenizer, tmp_path):
    """sahajBERT streaming semantics: sources mixed by probability through a shuffle buffer, each
    source restarting when exhausted (the stream never ends), deterministic per seed."""
    from dedloc_amd.data.sop_dataset import StreamingSOPStream

    tok, _ = tokenizer
    (tmp_path / "a.txt").write_text("\n\n".join(_corpus(5, seed=2)) + "\n")
    (tmp_path / "b.txt").write_text("\n\n".join(_corpus(7, seed=3)) + "\n")
    srcs = [(str(tmp_path / "a.txt"), 0.23), (str(tmp_path / "b.txt"), 0.77)]

    def make(seed):
        return StreamingSOPStream(srcs, tok, batch_size=4, seed=seed, max_seq_length=48, shuffle_buffer=16)

    s = make(3)
    batches = [s.next_batch() for _ in range(60)]  # far more instances than the 12 documents hold
    for b in batches:
        assert b["input_ids"].shape[0] == 4 and b["input_ids"].shape[1] <= 48
        assert set(b["sentence_order_label"].tolist()) <= {0, 1}
        assert ((b["labels"] == -100) | b["attention_mask"].bool()).all()
    frac = s.source_counts[0] / sum(s.source_counts)
    assert sum(s.source_counts) > 24 and 0.1 < frac < 0.38
    again = make(3)
    assert all(torch.equal(again.next_batch()["input_ids"], batches[i]["input_ids"]) for i in range(5))
    other = make(4)
    assert not all(torch.equal(other.next_batch()["input_ids"], batches[i]["input_ids"]) for i in range(5))


@pytest.mark.timeout(300)
def test_run_trainer_streaming_sources(tokenizer, tmp_path):
    """run_trainer --stream_sources: the sahajBERT streaming path (tokenizer from --tokenizer_path,
    embeddings resized to it) trains a peer for two collaborative steps."""
    from dedloc_amd.dht import DHT
    from dedloc_amd.models.albert import AlbertConfig

    tok, tok_dir = tokenizer
    (tmp_path / "w.txt").write_text("\n\n".join(_corpus(20, seed=4)) + "\n")
    (tmp_path / "o.txt").write_text("\n\n".join(_corpus(30, seed=5)) + "\n")
    cfgdir = tmp_path / "cfg"
    AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64).save_pretrained(str(cfgdir))
    root = DHT(listen_on="127.0.0.1:*")
    try:
        metrics = tmp_path / "m.jsonl"
        cmd = [sys.executable, "-m", "dedloc_amd.cli.run_trainer", "--experiment_prefix", "stream",
               "--initial_peers", root.endpoint, "--device", "cpu", "--config_path", str(cfgdir),
               "--stream_sources", f"{tmp_path / 'w.txt'}:0.23,{tmp_path / 'o.txt'}:0.77",
               "--tokenizer_path", tok_dir, "--seq_length", "64", "--per_device_train_batch_size", "2",
               "--gradient_accumulation_steps", "1", "--target_batch_size", "4", "--stop_after_global_steps", "2",
               "--save_steps", "0", "--output_dir", str(tmp_path / "out"), "--min_refresh_period", "0.05",
               "--default_refresh_period", "0.1", "--dht_listen_on", "127.0.0.1:*", "--listen_on", "127.0.0.1:*",
               "--metrics_file", str(metrics)]
        env = dict(os.environ, PYTHONPATH=ROOT)
        env.pop("RANK", None)
        env.pop("WORLD_SIZE", None)
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        assert "streaming SOP instances" in r.stderr
        recs = [json.loads(x) for x in metrics.read_text().splitlines()]
        assert max(rec["step"] for rec in recs) >= 2 and all(torch.isfinite(torch.tensor(rec["loss"])) for rec in recs)
    finally:
        root.shutdown()
