"""Host time to ISSUE one in-process multi-device round (bench.py's
`inprocess` step: reduce_into on every shard of a MultiDeviceBucket, no
sync), against the per-device kernel time it has to hide behind.  On N real
GPUs the last device starts its kernel only after the host has issued the
other N-1 shards, so issue time per shard x N must stay well below one
shard's kernel time.  Shards share one GPU here; only the host side is
measured.  Config 3's layout at 128 clients."""
from __future__ import annotations

import json
import time

import torch

from fedml_amd import multidev
from fedml_amd.shapes import resnet50


def main():
    dev = torch.device("cuda", 0)
    entries = resnet50()
    K = 128
    out = {}
    for G, batched in [(g, b) for g in (1, 2, 4, 8) for b in (False, True)]:
        mb = multidev.MultiDeviceBucket(entries, K, [dev] * G)
        outs = [b.new_outputs() for b in mb.shards]
        w = mb.weights([100 + i for i in range(K)])

        def step_each():
            for s, b in enumerate(mb.shards):
                b.reduce_into(outs[s], w)

        def step_batch():
            assert mb.reduce_into_all(outs, w)

        step = step_batch if batched else step_each

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        issue = []
        for _ in range(20):
            t0 = time.perf_counter()
            step()
            issue.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
        issue.sort()
        out[f"{G}{' batched' if batched else ''}"] = {"issue_us_median": round(issue[len(issue) // 2] * 1e6, 1),
                  "per_shard_us": round(issue[len(issue) // 2] * 1e6 / G, 1),
                  "launches_per_shard": [sum(1 for g in b.groups.values() if g.length) for b in mb.shards]}
        print(G, "batched" if batched else "each", out[f"{G}{' batched' if batched else ''}"], flush=True)
        del mb, outs
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
