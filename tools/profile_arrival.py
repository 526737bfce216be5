"""cProfile of the cross-silo arrival path (tool, GPU only): one warm round,
then one profiled round of add_local_trained_result for a bench config."""
from __future__ import annotations

import argparse
import cProfile
import os
import pstats
import sys
import time
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import bench  # noqa: E402
from e2e_configs import _Args, make_updates  # noqa: E402
from fedml_amd import shapes  # noqa: E402
from fedml_amd.cross_silo import FedMLAggregator  # noqa: E402
from fedml_amd.server_aggregator import MI355XServerAggregator  # noqa: E402
from fedml_amd.synth import sample_nums  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg5")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS[a.config]
    entries = shapes.MODELS[cfg["model"]]()
    K = cfg["K"]
    ups = make_updates(entries, 8, dev)
    ns = sample_nums(K)
    args = _Args()
    agg = MI355XServerAggregator(torch.nn.Linear(1, 1), args)
    agg.set_model_params = lambda p: None
    server = FedMLAggregator(None, None, 0, {}, {}, {}, K, dev, args, agg)

    def round_():
        for i in range(K):
            server.add_local_trained_result(i, OrderedDict(ups[i % 8]), ns[i])
        server.check_whether_all_receive()
        server.aggregate()
        torch.cuda.synchronize()

    round_()
    round_()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for i in range(K):
        server.add_local_trained_result(i, OrderedDict(ups[i % 8]), ns[i])
    pr.disable()
    torch.cuda.synchronize()
    print(f"{K} arrivals: {(time.perf_counter() - t0) * 1e3:.2f} ms (profiled)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
