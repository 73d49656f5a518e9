"""Decentralized averaging: matchmaking, LP load balancing, butterfly all-reduce over RCCL, state sharing."""
from .allreduce import AllreduceException, GroupSpec, butterfly_allreduce
from .averager import DecentralizedAverager
from .load_balancing import hagenbach_bischoff, load_balance_peers, optimize_parts_lp

__all__ = ["AllreduceException", "GroupSpec", "butterfly_allreduce", "DecentralizedAverager", "hagenbach_bischoff",
           "load_balance_peers", "optimize_parts_lp"]
