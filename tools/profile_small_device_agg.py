"""cProfile of agg() on config 1's device dicts (4 clients x 7,850 fp32):
where the ~58 us per call go (round 5).  Run from the repo root."""
from __future__ import annotations

import cProfile
import pstats
import sys
import time
from collections import OrderedDict

sys.path.insert(0, ".")
import torch  # noqa: E402

from fedml_amd.agg_operator import FedMLAggOperator  # noqa: E402


class _Args:
    federated_optimizer = "FedAvg"


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    base = [OrderedDict(w=torch.randn(10, 784, generator=g, device=dev), b=torch.randn(10, generator=g, device=dev))
            for _ in range(4)]

    def one():
        raw = [(100 + i, OrderedDict(d)) for i, d in enumerate(base)]
        FedMLAggOperator.agg(_Args(), raw)

    for _ in range(200):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2000):
        one()
    torch.cuda.synchronize()
    print(f"agg() on config-1 device dicts: {(time.perf_counter() - t0) / 2000 * 1e6:.1f} us per call", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(2000):
        one()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
