"""Downstream fine-tuning heads and recipe (reference sahajbert/train_ner.py,
sahajbert/train_ncc.py): HF key/logit parity of the classification heads with ``transformers``,
loading a pre-training checkpoint into a head model, the BIO span metric, and the fine-tuning loop
(early stopping, best-model restore) on synthetic task data."""
import json

import pytest
import torch

from dedloc_amd.cli import finetune
from dedloc_amd.models.albert import (AlbertConfig, AlbertForPreTraining, AlbertForSequenceClassification,
                                      AlbertForTokenClassification)


def _cfg():
    return AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64, classifier_dropout_prob=0.0)


@pytest.mark.parametrize("ours_cls,hf_name", [(AlbertForSequenceClassification, "AlbertForSequenceClassification"),
                                              (AlbertForTokenClassification, "AlbertForTokenClassification")])
def test_heads_match_transformers(tmp_path, ours_cls, hf_name):
    import transformers

    torch.manual_seed(0)
    ours = ours_cls(_cfg(), num_labels=5)
    ours.save_pretrained(str(tmp_path))
    hf = getattr(transformers, hf_name).from_pretrained(str(tmp_path)).eval()
    assert set(hf.state_dict()) >= set(ours.hf_state_dict()), "key mismatch"
    assert hf.config.num_labels == 5
    ours.materialize("cpu")
    ours.eval()
    ids = torch.randint(5, 500, (2, 64))
    mask = torch.ones_like(ids)
    mask[1, 40:] = 0
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=mask).logits
    got = ours(ids, mask)["logits"].float()
    if ours_cls is AlbertForTokenClassification:  # compare real tokens only
        keep = mask.bool()
        got, ref = got[keep], ref[keep]
    assert ((got - ref).norm() / ref.norm()).item() < 3e-2


def test_head_loads_pretraining_checkpoint(tmp_path):
    torch.manual_seed(1)
    pre = AlbertForPreTraining(_cfg())
    pre.save_pretrained(str(tmp_path))
    tok = AlbertForTokenClassification.from_pretrained(str(tmp_path), num_labels=7)
    a = pre.hf_state_dict()["albert.encoder.embedding_hidden_mapping_in.weight"]
    b = tok.hf_state_dict()["albert.encoder.embedding_hidden_mapping_in.weight"]
    assert torch.equal(a, b) and tok.num_labels == 7
    assert "albert.pooler.weight" not in tok.hf_state_dict()  # HF token classifier has no pooler
    seq = AlbertForSequenceClassification.from_pretrained(str(tmp_path), num_labels=3)
    assert torch.equal(seq.hf_state_dict()["albert.pooler.weight"], pre.hf_state_dict()["albert.pooler.weight"])


def test_bio_span_metric():
    refs = [["O", "B-PER", "I-PER", "O", "B-LOC"], ["B-ORG", "I-ORG", "O"]]
    preds = [["O", "B-PER", "I-PER", "O", "B-ORG"], ["B-ORG", "I-ORG", "O"]]
    m = finetune.ner_metrics(preds, refs)
    assert m["precision"] == pytest.approx(2 / 3) and m["recall"] == pytest.approx(2 / 3)
    assert m["accuracy"] == pytest.approx(7 / 8)
    # an I- tag that starts a span counts as an entity (IOB2 / seqeval default)
    assert finetune._spans(["I-LOC", "I-LOC", "O"]) == {(0, 2, "LOC")}


@pytest.mark.parametrize("task", ["ncc", "ner"])
def test_finetune_recipe_learns_cpu(tmp_path, task):
    args = finetune.parse_args(["--task", task, "--train_samples", "256", "--eval_samples", "64",
                                "--num_train_epochs", "3", "--max_seq_length", "64", "--learning_rate", "1e-3",
                                "--output_dir", str(tmp_path), "--early_stopping_patience", "3"])
    res = finetune.run(args)
    first = res["history"][0]
    assert res["history"][-1]["eval_loss"] < first["eval_loss"]
    key = "test_accuracy"
    assert res[key] > (1 / 6 + 0.1 if task == "ncc" else 0.7), res
    saved = json.load(open(tmp_path / "all_results.json"))
    assert saved["task"] == task
    assert (tmp_path / "pytorch_model.bin").exists()


def test_finetune_early_stopping_restores_best(monkeypatch):
    args = finetune.parse_args(["--task", "ncc", "--train_samples", "32", "--eval_samples", "16",
                                "--num_train_epochs", "6", "--max_seq_length", "64", "--learning_rate", "0.0",
                                "--early_stopping_patience", "2"])
    res = finetune.run(args)  # lr 0: the loss never improves after epoch 1 -> stop after 1 + patience epochs
    assert res["epochs_run"] == 3


@pytest.mark.gpu
def test_finetune_heads_gpu(cuda):
    args = finetune.parse_args(["--task", "ner", "--train_samples", "64", "--eval_samples", "32",
                                "--num_train_epochs", "2", "--max_seq_length", "128", "--learning_rate", "1e-3",
                                "--device", "cuda"])
    res = finetune.run(args)
    assert res["history"][-1]["eval_loss"] < res["history"][0]["eval_loss"] + 0.5
    assert res["test_accuracy"] > 0.5


def test_builtin_albert_configs():
    """Built-in config for albert-base-v2 next to albert-large-v2 (the model card's sizes and ~11.7M
    parameters); the reference-style URL maps to the built-in copy."""
    from dedloc_amd.models.albert import AlbertConfig, AlbertForPreTraining

    base = AlbertConfig.from_pretrained("https://s3.amazonaws.com/models.huggingface.co/bert/albert-base-v2-config.json")
    assert (base.hidden_size, base.num_hidden_layers, base.num_attention_heads, base.intermediate_size,
            base.embedding_size, base.vocab_size) == (768, 12, 12, 3072, 128, 30000)
    assert AlbertConfig.from_pretrained("albert-base-v2") == base
    m = AlbertForPreTraining(base)
    m.materialize("cpu")
    n = m.flat.fp32.numel()  # the tied decoder counted once, like HF
    assert 11.0e6 < n < 12.5e6, n
    xl = AlbertConfig.from_pretrained("albert-xlarge-v2")
    assert (xl.hidden_size, xl.num_hidden_layers, xl.num_attention_heads, xl.intermediate_size,
            xl.embedding_size) == (2048, 24, 16, 8192, 128)
    m = AlbertForPreTraining(xl)
    m.materialize("cpu")
    assert 57e6 < m.flat.fp32.numel() < 61e6  # the model card's ~59M
    del m
    import transformers

    xxl, hf = AlbertConfig.from_pretrained("albert-xxlarge-v2"), transformers.AlbertConfig()
    for k in ("vocab_size", "embedding_size", "hidden_size", "num_hidden_layers", "num_attention_heads",
              "intermediate_size", "num_hidden_groups", "inner_group_num"):
        assert getattr(xxl, k) == getattr(hf, k), k
