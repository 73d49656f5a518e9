"""Host-side cost of the SwAV peer's iteration: wall time of each train_step call (the host enqueues;
the GPU runs behind) and how far ahead of the GPU the host gets.  A host that is close to the GPU's
iteration time makes any GIL holder or host sync visible in the throughput."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dedloc_amd.dht import DHT  # noqa: E402
from dedloc_amd.training.swav_peer import SwavPeer  # noqa: E402
from dedloc_amd.utils.config import load_config  # noqa: E402


def main():
    n = int(os.environ.get("ITERS", "60"))
    cfg = load_config("swav_1node_resnet_submit", ["config.OPTIMIZER.target_batch_size=100000000",
                                                    "config.CHECKPOINT.DIR=/tmp/swav_host_probe"])
    dht = DHT(start=True)
    peer = SwavPeer(cfg, torch.device("cuda", 0), dht=dht)
    try:
        for _ in range(6):
            peer.train_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        host = []
        for _ in range(n):
            t = time.perf_counter()
            peer.train_step()
            host.append((time.perf_counter() - t) * 1e3)
        t_enq = time.perf_counter()
        torch.cuda.synchronize()
        t_end = time.perf_counter()
        host.sort()
        print(json.dumps({"iters": n, "wall_ms_per_iter": (t_end - t0) / n * 1e3,
                          "host_ms_median": host[n // 2], "host_ms_p90": host[int(n * 0.9)], "host_ms_max": host[-1],
                          "host_lead_ms_at_end": (t_end - t_enq) * 1e3}))
    finally:
        peer.shutdown()
        dht.shutdown()


if __name__ == "__main__":
    main()
