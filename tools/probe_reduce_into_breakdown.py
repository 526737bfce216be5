import time, torch, sys
sys.path.insert(0, '.')
from fedml_amd import multidev, kernels as kn
from fedml_amd.shapes import resnet50
dev = torch.device("cuda", 0)
mb = multidev.MultiDeviceBucket(resnet50(), 128, [dev] * 8)
b = mb.shards[0]; outs = b.new_outputs(); w = mb.weights([100 + i for i in range(128)])
g = b.groups[torch.float32]
def t(name, fn, n=2000):
    for _ in range(50): fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n): fn()
    dt = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    print(f"{name:40s} {dt:7.2f} us", flush=True)
hw = kn.weights_for(w, torch.float32, dev)
t("weights_for(128)", lambda: kn.weights_for(w, torch.float32, dev))
def ctx():
    with torch.cuda.device(dev): pass
t("with torch.cuda.device", ctx)
t("current_stream(dev)", lambda: torch.cuda.current_stream(dev))
cur = torch.cuda.current_stream(dev)
def sctx():
    with torch.cuda.stream(cur): pass
t("with torch.cuda.stream(cur)", sctx)
t("sync_ingest", b.sync_ingest)
t("dominant_dtype", b.dominant_dtype)
t("stream_handle", lambda: __import__('fedml_amd._native', fromlist=['x']).stream_handle())
t("wsum_ptrs (launch)", lambda: kn.wsum_ptrs(torch.float32, g.d_ptrs, hw, 128, g.length, outs[torch.float32], True), n=300)
t("reduce_into", lambda: b.reduce_into(outs, w), n=300)
