"""Probe: how much of the SwAV trunk forward's two resolution passes (2x224 crops, 6x96 crops of a
b=64 batch) could overlap on two HIP streams.  Times each pass alone, both back to back on one
stream, and both on two streams (forward only, training-mode BN; the running-statistics updates of
the two passes race in the concurrent arm, so it is a timing probe, not a training path)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401
from dedloc_amd.models.resnet_swav import SwAVModel  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = SwAVModel().to(dev).to(memory_format=torch.channels_last).train()
    cl = torch.channels_last
    x224 = torch.randn(128, 3, 224, 224, device=dev).bfloat16().contiguous(memory_format=cl)
    x96 = torch.randn(384, 3, 96, 96, device=dev).bfloat16().contiguous(memory_format=cl)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def p224():
        m.set_bn_stat_groups(2)
        return m.trunk(x224)

    def p96():
        m.set_bn_stat_groups(6)
        return m.trunk(x96)

    def seq():
        p224()
        p96()

    def conc():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            p224()
        with torch.cuda.stream(s2):
            p96()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    streams = [torch.cuda.Stream() for _ in range(4)]

    def multi(parts):  # parts: [(x, groups)] each on its own stream
        def run():
            cur = torch.cuda.current_stream()
            for st in streams[:len(parts)]:
                st.wait_stream(cur)
            for st, (x, g) in zip(streams, parts):
                m.set_bn_stat_groups(g)
                with torch.cuda.stream(st):
                    m.trunk(x)
            for st in streams[:len(parts)]:
                cur.wait_stream(st)
        return run

    x224a, x224b = x224[:64].contiguous(memory_format=cl), x224[64:].contiguous(memory_format=cl)
    x96a, x96b = x96[:192].contiguous(memory_format=cl), x96[192:].contiguous(memory_format=cl)
    with torch.no_grad():
        res = {"p224_ms": timeit(p224), "p96_ms": timeit(p96), "seq_ms": timeit(seq), "two_streams_ms": timeit(conc),
               "three_224split_ms": timeit(multi([(x224a, 1), (x224b, 1), (x96, 6)])),
               "three_96split_ms": timeit(multi([(x224, 2), (x96a, 3), (x96b, 3)])),
               "four_ms": timeit(multi([(x224a, 1), (x224b, 1), (x96a, 3), (x96b, 3)]))}
    print(json.dumps({k: round(v, 3) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
