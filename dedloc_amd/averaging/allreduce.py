"""Butterfly all-reduce over the RCCL (GPU) / gloo (CPU) world communicator.

A matchmade group (any subset of the world) averages a list of flat fp32 tensors:

  1. pack   : wire = compress(x * w_me)                    (one HIP pack kernel per tensor)
  2. scatter: member j receives part j of everyone's wire  (grouped isend/irecv, all pairs at once —
              on an 8-GPU xGMI mesh every GPU drives its 7 links concurrently instead of the one
              link per hop of a ring)
  3. reduce : avg_j = sum_k wire_k[j] / sum_k w_k          (HIP reduce kernel, fp32 accumulation)
  4. gather : every member receives every averaged part    (grouped isend/irecv)
  5. unpack : x = decompress(avg)  or the delta rule  x += decompress(avg) - snapshot

Part sizes come from the load-balancing LP; client-mode members own no part (they only send and
receive), auxiliary members contribute no tensor (weight 0) but reduce a part.  Because only the
group's ranks post operations, subsets need no extra communicators.
"""
from __future__ import annotations

import datetime
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

WIRE_DTYPES = {"NONE": torch.float32, "FLOAT32": torch.float32, "FLOAT16": torch.float16,
               "BFLOAT16": torch.bfloat16}


class AllreduceException(RuntimeError):
    pass


@dataclass
class GroupSpec:
    ranks: List[int]            # process-group rank of each member, in group order
    part_sizes: List[int]       # elements of the averaged vector owned by each member
    weights: List[float]        # averaging weight of each member (0 for auxiliary peers)
    contributes: List[bool]     # False for auxiliary peers (they send no tensor)
    my_index: int

    @property
    def size(self):
        return len(self.ranks)


def butterfly_allreduce(tensors: Sequence[torch.Tensor], spec: GroupSpec, compression: str = "FLOAT16",
                        pg=None, timeout: Optional[float] = 30.0, snapshots: Optional[Sequence[torch.Tensor]] = None,
                        sources: Optional[Sequence[torch.Tensor]] = None):
    """Average ``tensors`` in place across the group described by ``spec``.

    ``sources``: pack these instead of ``tensors`` (same shapes) — used by delayed parameter
    averaging, which averages a snapshot while the live parameters keep training.
    ``snapshots``: delta rule on unpack (``t += avg - snapshot``)."""
    ops = torch.ops.dedloc
    wire = WIRE_DTYPES[compression]
    dev = tensors[0].device
    sizes = [t.numel() for t in tensors]
    V = sum(sizes)
    assert sum(spec.part_sizes) == V, "part sizes must cover the averaged vector"
    me = spec.my_index
    starts = [0]
    for p in spec.part_sizes:
        starts.append(starts[-1] + p)
    my_lo, my_hi = starts[me], starts[me + 1]
    P = my_hi - my_lo
    total_w = float(sum(w for w, c in zip(spec.weights, spec.contributes) if c))
    if total_w <= 0:
        raise AllreduceException("group has no contributing weight")

    # 1. pack (weight-scaled, compressed) into one contiguous wire buffer
    send = torch.empty(V, dtype=wire, device=dev)
    if spec.contributes[me]:
        o = 0
        for t, n in zip(sources if sources is not None else tensors, sizes):
            ops.pack(t.reshape(-1), send[o:o + n], float(spec.weights[me]))
            o += n
    contrib_idx = [j for j in range(spec.size) if spec.contributes[j]]
    recv = torch.empty((max(1, len(contrib_idx)), max(P, 1)), dtype=wire, device=dev)

    def _run(p2p):
        if not p2p:
            return
        works = dist.batch_isend_irecv(p2p)
        td = datetime.timedelta(seconds=timeout) if timeout else None
        for w in works:
            if td is not None:
                if not w.wait(timeout=td):
                    raise AllreduceException("all-reduce timed out")
            else:
                w.wait()

    # 2. reduce-scatter
    p2p = []
    for slot, j in enumerate(contrib_idx):
        if j == me:
            if P:
                recv[slot, :P].copy_(send[my_lo:my_hi])
            continue
        if P:
            p2p.append(dist.P2POp(dist.irecv, recv[slot, :P], spec.ranks[j], group=pg))
    if spec.contributes[me]:
        for j in range(spec.size):
            if j != me and spec.part_sizes[j] > 0:
                p2p.append(dist.P2POp(dist.isend, send[starts[j]:starts[j + 1]], spec.ranks[j], group=pg))
    _run(p2p)

    # 3. reduce my part (fp32 accumulation, weighted mean), result in wire dtype
    gathered = send  # reuse: everyone's averaged parts land here
    if P:
        avg = torch.empty(P, dtype=wire, device=dev)
        part_view = recv[:, :P].contiguous() if recv.shape[1] != P else recv
        ops.reduce_parts(part_view, len(contrib_idx), avg, 1.0 / total_w)
        gathered[my_lo:my_hi].copy_(avg)

    # 4. all-gather of the averaged parts
    p2p = []
    for j in range(spec.size):
        if j == me:
            continue
        if P:
            p2p.append(dist.P2POp(dist.isend, gathered[my_lo:my_hi], spec.ranks[j], group=pg))
        if spec.part_sizes[j] > 0:
            p2p.append(dist.P2POp(dist.irecv, gathered[starts[j]:starts[j + 1]], spec.ranks[j], group=pg))
    _run(p2p)

    # 5. unpack (auxiliary peers keep their buffers untouched unless they hold tensors)
    o = 0
    for k, (t, n) in enumerate(zip(tensors, sizes)):
        snap = None if snapshots is None else snapshots[k].reshape(-1)
        ops.unpack(gathered[o:o + n], t.reshape(-1), snap)
        o += n
    return total_w
