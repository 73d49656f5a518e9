"""Per-GPU emulation of the reference's heterogeneous, churning volunteer fleet (SURVEY.md §2.1 D9/D15,
§5.3): the AWS runner (``albert/AWS_runner.ipynb``) mixes T4 spot workers with 200/100/50 Mbps
``wondershaper`` caps, CPU auxiliary peers and a preemption-respawn loop; sahajBERT volunteers join
with micro-batches of 1-4 and leave at will.  On one MI355X node every peer is a GPU process, so the
heterogeneity is injected: per-rank micro-batch, compute slowdown / throttle, emulated bandwidth
(fed to the load-balancing LP, optionally also as transfer delay), client mode, and a churn schedule
that takes a peer out of the collaboration (leave) or makes it lose its state and rejoin (restart).
"""
from .churn import ChurnController, ChurnEvent, parse_churn_schedule
from .heterogeneity import PeerProfile, StepThrottle, aws_fleet_profiles, profile_for_rank, select_for_rank

__all__ = ["ChurnController", "ChurnEvent", "parse_churn_schedule", "PeerProfile", "StepThrottle",
           "aws_fleet_profiles", "profile_for_rank", "select_for_rank"]
