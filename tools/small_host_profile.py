"""cProfile of FedMLAggOperator.agg on host dicts at configs 1 and 2 (where
fixed per-call costs dominate): which host-side steps the ~0.1-0.6 ms go to.
Writes gpurun_out/small_host_profile_<cfg>.txt.

    python tools/small_host_profile.py
"""
from __future__ import annotations

import cProfile
import io
import os
import pstats
import sys
from collections import OrderedDict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedml_amd import shapes  # noqa: E402
from fedml_amd.agg_operator import FedMLAggOperator  # noqa: E402
from fedml_amd.synth import host_clients  # noqa: E402


class _Args:
    federated_optimizer = "FedAvg"


def main():
    os.makedirs("gpurun_out", exist_ok=True)
    args = _Args()
    for cfg, model, K in (("cfg1", "lr_mnist", 4), ("cfg2", "cnn_web", 32)):
        raw = host_clients(shapes.MODELS[model](), K, seed=1)
        for _ in range(20):
            FedMLAggOperator.agg(args, [(n, OrderedDict(d)) for n, d in raw])
        torch.cuda.synchronize()
        lists = [[(n, OrderedDict(d)) for n, d in raw] for _ in range(300)]
        pr = cProfile.Profile()
        pr.enable()
        for lst in lists:
            FedMLAggOperator.agg(args, lst)
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        with open(f"gpurun_out/small_host_profile_{cfg}.txt", "w") as f:
            f.write(s.getvalue())
        print(cfg, s.getvalue()[:3000])


if __name__ == "__main__":
    main()
