"""Flag surface of the reference entry points (albert/arguments.py:7-128, run_first_peer.py:24-56,
SURVEY.md App. B) plus the MI355X emulation knobs.  Parsed with
``transformers.HfArgumentParser`` exactly like the reference (``--flag value``; lists are
space-separated, e.g. ``--initial_peers a:1 b:2``)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class BaseTrainingArguments:
    experiment_prefix: str = field(metadata={"help": "A unique 'name' of this experiment, used to store metadata on the DHT"})
    initial_peers: List[str] = field(default_factory=list,
                                     metadata={"help": "One or more peers that will welcome you into the collaboration"})
    dht_listen_on: str = field(default="[::]:*", metadata={"help": "Network interface used for incoming DHT communication"})


@dataclass
class AveragerArguments:
    averaging_expiration: float = field(default=5.0, metadata={"help": "Averaging group will wait for stragglers for at most this many seconds"})
    averaging_timeout: float = field(default=30.0, metadata={"help": "Give up on averaging step after this many seconds"})
    listen_on: str = field(default="[::]:*", metadata={"help": "Network interface used for incoming averager communication"})
    min_refresh_period: float = field(default=0.5, metadata={"help": "Wait for at least this many seconds before fetching new collaboration state"})
    max_refresh_period: float = field(default=30, metadata={"help": "Wait for at most this many seconds before fetching new collaboration state"})
    default_refresh_period: float = field(default=3, metadata={"help": "Attempt to fetch collaboration state every this often until successful"})
    expected_drift_peers: float = field(default=3, metadata={"help": "Trainer assumes that this many new peers can join per step"})
    expected_drift_rate: float = field(default=0.2, metadata={"help": "Trainer assumes that this fraction of current size can join per step"})
    performance_ema_alpha: float = field(default=0.1, metadata={"help": "Uses this alpha for moving average estimate of samples per second"})
    target_group_size: int = field(default=256, metadata={"help": "Maximum group size for all-reduce"})
    metadata_expiration: float = field(default=30, metadata={"help": "Peer's metadata will be removed if not updated in this many seconds"})


@dataclass
class CollaborativeOptimizerArguments:
    target_batch_size: int = field(default=4096, metadata={"help": "Perform optimizer step after all peers collectively accumulate this many samples"})
    client_mode: bool = field(default=False, metadata={"help": "If True, runs training without incoming connections"})
    batch_size_lead: int = field(default=0, metadata={"help": "Optional: begin looking for group in advance, this many samples before target_batch_size"})
    bandwidth: float = field(default=100.0, metadata={"help": "Available network bandwidth, in mbps (used for load balancing in all-reduce)"})
    compression: str = field(default="FLOAT16", metadata={"help": "Use this compression when averaging parameters/gradients (NONE, FLOAT16, BFLOAT16)"})


@dataclass
class CollaborationArguments(AveragerArguments, CollaborativeOptimizerArguments, BaseTrainingArguments):
    statistics_expiration: float = field(default=600, metadata={"help": "Statistics will be removed if not updated in this many seconds"})
    endpoint: Optional[str] = field(default=None, metadata={"help": "This node's IP for inbound connections"})
    # ---- MI355X additions: fault-tolerance path and bandwidth emulation
    delay_param_averaging: bool = field(default=False, metadata={"help": "average gradients synchronously but parameters in the background (delta rule)"})
    peer_bandwidths: Optional[str] = field(default=None, metadata={"help": "per-rank emulated bandwidth list (Mbps), e.g. 200,100,100,50"})
    peer_client_mode: Optional[str] = field(default=None, metadata={"help": "per-rank client-mode flags, e.g. 0,0,0,1"})
    emulate_transfer_delay: bool = field(default=False, metadata={"help": "also delay each all-reduce to the emulated bandwidth's transfer time"})
    eta_slack: float = field(default=0.5, metadata={
        "help": "begin the global step when the collaboration's ETA falls within this fraction of one local step "
                "from now (0 = hivemind's rule: only once the ETA has passed)"})


@dataclass
class DatasetArguments:
    dataset_path: Optional[str] = field(default="data/albert_tokenized_wikitext", metadata={"help": "Path to the tokenized dataset (synthetic if absent)"})
    tokenizer_path: Optional[str] = field(default="data/tokenizer", metadata={"help": "Path to the tokenizer"})
    config_path: Optional[str] = field(default="https://s3.amazonaws.com/models.huggingface.co/bert/albert-large-v2-config.json",
                                       metadata={"help": "Path to the model config (the albert-large-v2 URL maps to the built-in config)"})
    cache_dir: Optional[str] = field(default="data", metadata={"help": "Path to the cache"})
    vocab_size: Optional[int] = field(default=None, metadata={"help": "Override the vocabulary size (sahajBERT: 31995)"})
    length_mode: str = field(default="full", metadata={"help": "synthetic instance lengths: full (all 512) or wikitext (10% short tails)"})
    mask_mode: str = field(default="fixed", metadata={"help": "fixed (max_predictions_per_seq form) or hf (Bernoulli 15%)"})
    stream_sources: Optional[str] = field(default=None, metadata={
        "help": "sahajBERT streaming corpus over local text: 'path_a:0.23,path_b:0.77' (tokenized on the fly "
                "with --tokenizer_path, 10^4-document shuffle buffer, per-peer seed)"})


@dataclass
class AlbertTrainingArguments:
    output_dir: str = "outputs"
    overwrite_output_dir: bool = False
    do_train: bool = True
    do_eval: bool = False
    per_device_train_batch_size: int = 4
    per_device_eval_batch_size: int = 4
    gradient_accumulation_steps: int = 2
    seq_length: int = 512
    max_steps: int = 1_000_000
    learning_rate: float = 0.00176
    warmup_steps: int = 5000
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_epsilon: float = 1e-6
    weight_decay: float = 0.01
    max_grad_norm: float = 1.0
    clamp_value: float = 10000.0
    fp16: bool = True
    fp16_opt_level: str = "O2"
    bf16: bool = True
    logging_dir: Optional[str] = None
    logging_first_step: bool = False
    logging_steps: int = 100
    save_total_limit: int = 2
    save_steps: int = 500
    seed: int = 42
    run_name: Optional[str] = None
    dataloader_num_workers: int = 4
    device: Optional[str] = None
    # ---- MI355X emulation of the reference's heterogeneous AWS fleet
    throttle: float = field(default=0.0, metadata={"help": "extra idle seconds per training step (emulates a slower peer)"})
    slowdown: float = field(default=1.0, metadata={"help": "emulate slower hardware: each step takes this many times longer"})
    churn_schedule: Optional[str] = field(default=None, metadata={"help": "drop-out/drop-in schedule '[leave|restart@]AT[s]:DURATION,...' (emulation/churn.py)"})
    peer_batch_sizes: Optional[str] = field(default=None, metadata={"help": "per-rank micro-batch list, e.g. 32,16,8,4 (cycled over ranks)"})
    peer_slowdowns: Optional[str] = field(default=None, metadata={"help": "per-rank slowdown list, e.g. 1,1.3,2"})
    peer_churn: Optional[str] = field(default=None, metadata={"help": "per-rank churn schedules separated by ';' (empty = none)"})
    stop_after_global_steps: Optional[int] = field(default=None, metadata={"help": "exit after this many collaborative steps"})
    metrics_file: Optional[str] = field(default=None, metadata={"help": "append per-global-step JSONL metrics here"})


@dataclass
class CoordinatorArguments(BaseTrainingArguments):
    address: Optional[str] = field(default=None, metadata={"help": "This machine's network address (127.0.0.1 on a single node)"})
    refresh_period: float = field(default=30, metadata={"help": "Coordinator will fetch keys from DHT once in this many seconds"})
    wandb_project: Optional[str] = field(default=None, metadata={"help": "Learning curves will be published there (needs network; off)"})
    save_checkpoint_step_interval: int = field(default=5, metadata={"help": "Coordinator will load and save state from peers once every that many steps"})
    model_config_path: str = field(default="https://s3.amazonaws.com/models.huggingface.co/bert/albert-large-v2-config.json",
                                   metadata={"help": "Path to the model config"})
    repo_path: Optional[str] = field(default=None, metadata={"help": "Directory (optionally a git repo) where the coordinator saves model + optimizer state"})
    upload_interval: Optional[float] = field(default=None, metadata={"help": "Coordinator will upload model once in this many seconds"})
    metrics_file: Optional[str] = field(default=None, metadata={"help": "append aggregated collaboration metrics here (JSONL)"})
    max_runtime: Optional[float] = field(default=None, metadata={"help": "exit after this many seconds"})
    device: Optional[str] = field(default="cpu", metadata={"help": "device for the coordinator's model replica"})
    vocab_size: Optional[int] = field(default=None, metadata={"help": "override the replica's vocabulary size (sahajBERT: 31995)"})
