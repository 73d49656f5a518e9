"""Tiny hierarchical config system with command-line overrides.

Replaces vissl's hydra composition (``tools/run_distributed_engines.py:21-58``,
``utils/hydra_config.py``) for the one config the collaborative SwAV run needs: a YAML file (read
with ``yaml.safe_load`` only) plus dotted overrides in the same spelling as the reference's launch
recipe (``swav/README.md:17-31``)::

    config=pretrain/swav/swav_1node_resnet_submit  config.DATA.TRAIN.BATCHSIZE_PER_REPLICA=64
    +config.OPTIMIZER.lr=2.4  +config.OPTIMIZER.dht_initial_peers=["1.2.3.4:1337"]

The ``+`` prefix (hydra's "add a new key") is accepted and ignored; values are parsed as YAML.
"""
from __future__ import annotations

import copy
from pathlib import Path
from typing import Any, Dict, Iterable, Optional

import yaml

CONFIG_DIR = Path(__file__).resolve().parent.parent / "configs"


class AttrDict(dict):
    """dict with attribute access (nested dicts are converted on construction)."""

    def __init__(self, d: Optional[Dict] = None):
        super().__init__()
        for k, v in (d or {}).items():
            self[k] = AttrDict(v) if isinstance(v, dict) and not isinstance(v, AttrDict) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = AttrDict(v) if isinstance(v, dict) and not isinstance(v, AttrDict) else v

    def get_path(self, dotted: str, default=None):
        cur: Any = self
        for part in dotted.split("."):
            if not isinstance(cur, dict) or part not in cur:
                return default
            cur = cur[part]
        return cur

    def to_dict(self) -> Dict:
        return {k: (v.to_dict() if isinstance(v, AttrDict) else copy.deepcopy(v)) for k, v in self.items()}


def _resolve(name: str) -> Path:
    p = Path(name)
    if p.suffix != ".yaml":
        p = p.with_suffix(".yaml")
    if p.exists():
        return p
    q = CONFIG_DIR / p
    if q.exists():
        return q
    q = CONFIG_DIR / p.name  # "pretrain/swav/swav_1node_resnet_submit" -> configs/swav_1node_resnet_submit.yaml
    if q.exists():
        return q
    raise FileNotFoundError(f"config {name!r} not found (looked in cwd and {CONFIG_DIR})")


def set_path(cfg: AttrDict, dotted: str, value):
    parts = dotted.split(".")
    cur = cfg
    for part in parts[:-1]:
        if part not in cur or not isinstance(cur[part], dict):
            cur[part] = AttrDict()
        cur = cur[part]
    cur[parts[-1]] = AttrDict(value) if isinstance(value, dict) else value


def load_config(name: str = "swav_1node_resnet_submit", overrides: Iterable[str] = ()) -> AttrDict:
    """Load a YAML config (top-level ``config:`` key) and apply ``[+]config.A.B=value`` overrides."""
    with open(_resolve(name)) as f:
        raw = yaml.safe_load(f) or {}
    cfg = AttrDict(raw.get("config", raw))
    for ov in overrides:
        key, sep, val = ov.partition("=")
        if not sep:
            raise ValueError(f"override {ov!r} is not KEY=VALUE")
        key = key.lstrip("+")
        if key.startswith("config."):
            key = key[len("config."):]
        set_path(cfg, key, yaml.safe_load(val) if val != "" else None)
    return cfg


def parse_cli(argv: Iterable[str]):
    """Split ``config=NAME`` from the override list (hydra-style positional arguments)."""
    name, overrides, rest = "swav_1node_resnet_submit", [], []
    for a in argv:
        if a.startswith("config="):
            name = a.partition("=")[2]
        elif "=" in a and (a.startswith("config.") or a.startswith("+config.")):
            overrides.append(a)
        else:
            rest.append(a)
    return name, overrides, rest
