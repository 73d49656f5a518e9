"""Butterfly all-reduce over a group communicator (RCCL on GPUs, gloo on CPU).

A matchmade group (any set of live peers) averages a list of flat fp32 tensors:

  1. pack   : wire = compress(x)                             (one HIP pack kernel per tensor)
  2. scatter: member j receives part j of everyone's wire    (one grouped send/recv, all pairs at once —
              on an 8-GPU xGMI mesh every GPU drives its 7 links concurrently instead of the one
              link per hop of a ring)
  3. reduce : avg_j = sum_k w_k wire_k[j] / sum_k w_k in fp32, and for every sender k the delta
              d_k[j] = compress(avg_j - decompress(wire_k[j]))     (one HIP reduce_delta kernel)
  4. return : member j sends d_k[j] back to sender k          (one grouped send/recv)
  5. unpack : x += decompress(d)                              (fp32, on the live tensor)

Returning averaged-part *deltas* (hivemind 0.9.x's ``averaged_part - tensor_part`` rule) instead of
the average keeps each peer's fp32 master tensor: the peer adds (average - what it sent), so the
compression residual of its own contribution stays in its fp32 tensor and parameter updates below
half a FLOAT16 ulp survive averaging (replacing the tensor by the decoded average would round the
master parameters to fp16 every global step).  When all peers hold the same tensor the deltas are
exactly zero.

Part sizes come from the load-balancing LP; client-mode members own no part (they only send and
receive), auxiliary members contribute no tensor (weight 0) but reduce a part.

Weights travel on the wire: each contributor sends its own fp32 weight (bit-exact, as 1-2 wire
elements) to every reducer together with the part, and the reducer reads the weights it applies
from what it received.  Only ``spec.weights[my_index]`` has to be known when the round starts — so
matchmaking can run ahead of the last micro-step of a global batch, before a peer knows how many
samples it will have contributed (``DecentralizedAverager.prejoin``) — and it may be a device scalar
(the count of finite samples, kept on the GPU), so the global step never waits for the host to
learn it.  A group whose weights sum to 0 leaves every tensor unchanged (zero deltas).

Timeouts: completion is polled on the host against a deadline; on expiry the communicator is
aborted (``ncclCommAbort`` for RCCL) so the operations still posted on it can never be matched by a
later round, and the round raises ``AllreduceException``; the caller drops the communicator from its
cache (``parallel.GroupCommunicators.invalidate``).
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from ..parallel.comm import CommError

WIRE_DTYPES = {"NONE": torch.float32, "FLOAT32": torch.float32, "FLOAT16": torch.float16,
               "BFLOAT16": torch.bfloat16}


class AllreduceException(CommError):
    pass


@dataclass
class GroupSpec:
    ranks: List[int]            # communicator rank of each member, in group order
    part_sizes: List[int]       # elements of the averaged vector owned by each member
    weights: List[float]        # averaging weight of each member (0 for auxiliary peers)
    contributes: List[bool]     # False for auxiliary peers (they send no tensor)
    my_index: int

    @property
    def size(self):
        return len(self.ranks)


def _p2p(comm, sends, send_peers, recvs, recv_peers, deadline, tag):
    if not sends and not recvs:
        return
    if comm is None:
        raise AllreduceException("a group of more than one member needs a communicator")
    try:
        comm.p2p(sends, send_peers, recvs, recv_peers, deadline, tag=tag)
    except CommError as e:
        raise AllreduceException(str(e)) from e


def butterfly_allreduce(tensors: Sequence[torch.Tensor], spec: GroupSpec, compression: str = "FLOAT16",
                        comm=None, timeout: Optional[float] = 30.0, sources: Optional[Sequence[torch.Tensor]] = None):
    """Average ``tensors`` in place across the group described by ``spec``.

    ``sources``: pack these instead of ``tensors`` (same shapes) and add the averaging deltas to
    ``tensors`` — delayed parameter averaging packs a snapshot and collects the delta in a zeroed
    buffer while the live parameters keep training."""
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
    contrib_idx = [j for j in range(spec.size) if spec.contributes[j]]
    if not contrib_idx:
        raise AllreduceException("group has no contributing member")
    deadline = time.monotonic() + timeout if timeout else None
    i_contribute = spec.contributes[me]
    # this contributor's weight as wire elements (the fp32 bits: 1 element of fp32, 2 of fp16/bf16)
    W = 4 // torch.empty(0, dtype=wire).element_size()
    w_me = spec.weights[me]
    if isinstance(w_me, torch.Tensor):  # a device scalar: the weight is never read on the host
        my_w = w_me.detach().reshape(1).to(device=dev, dtype=torch.float32).contiguous().view(wire)
    else:
        my_w = torch.tensor([float(w_me)], dtype=torch.float32).view(wire).to(dev)

    # 1. pack (compressed, unweighted: the reducer applies the weights in fp32)
    send = torch.empty(V if i_contribute else 0, dtype=wire, device=dev)
    if i_contribute:
        o = 0
        for t, n in zip(sources if sources is not None else tensors, sizes):
            ops.pack(t.reshape(-1), send[o:o + n], 1.0)
            o += n
    nc = len(contrib_idx)
    recv = torch.empty((max(1, nc), max(P, 1)), dtype=wire, device=dev)
    wrecv = torch.empty((max(1, nc), W), dtype=wire, device=dev)

    # 2. reduce-scatter: part j of every contributor's wire (and its weight) goes to member j (one
    #    grouped launch; the two transfers of a pair are matched in order)
    sends, send_peers, recvs, recv_peers = [], [], [], []
    for slot, j in enumerate(contrib_idx):
        if j == me:
            if P:
                recv[slot, :P].copy_(send[my_lo:my_hi])
                wrecv[slot].copy_(my_w)
            continue
        if P:
            recvs += [recv[slot, :P], wrecv[slot]]
            recv_peers += [spec.ranks[j]] * 2
    if i_contribute:
        for j in range(spec.size):
            if j != me and spec.part_sizes[j] > 0:
                sends += [send[starts[j]:starts[j + 1]], my_w]
                send_peers += [spec.ranks[j]] * 2
    _p2p(comm, sends, send_peers, recvs, recv_peers, deadline, tag=1)

    # 3. weighted fp32 average of my part and one delta row per contributor
    deltas = None
    if P:
        parts = recv if recv.shape[1] == P else recv[:, :P].contiguous()
        w = wrecv.view(torch.float32).reshape(-1)
        deltas = torch.empty_like(parts)
        ops.reduce_delta(parts, w, deltas)

    # 4. every contributor receives its deltas for every part
    dbuf = torch.empty(V if i_contribute else 0, dtype=wire, device=dev)
    sends, send_peers, recvs, recv_peers = [], [], [], []
    for slot, j in enumerate(contrib_idx):
        if j == me:
            if P:
                dbuf[my_lo:my_hi].copy_(deltas[slot])
            continue
        if P:
            sends.append(deltas[slot])
            send_peers.append(spec.ranks[j])
    if i_contribute:
        for j in range(spec.size):
            if j != me and spec.part_sizes[j] > 0:
                recvs.append(dbuf[starts[j]:starts[j + 1]])
                recv_peers.append(spec.ranks[j])
    _p2p(comm, sends, send_peers, recvs, recv_peers, deadline, tag=2)

    # 5. unpack: x += delta (auxiliary peers hold no averaged tensor)
    if i_contribute:
        o = 0
        for t, n in zip(tensors, sizes):
            ops.unpack(dbuf[o:o + n], t.reshape(-1), None, True)
            o += n
