"""A/B of the fused forward kernel with and without the saved product (want_P: the training
forward also stores A Z_k for the backward), V4 m=256 n=512 K=15 B=65,536, interleaved in one
process, HIP-event kernel times (median of 10).  Prints one JSON line."""
import os, sys, importlib, json, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); import bench
dl = importlib.import_module("d-ladmm_amd"); ops = importlib.import_module("d-ladmm_amd.ops")
dev = torch.device("cuda", 0); m, n, K, B = 256, 512, 15, 65536
A, X, Z0, E0, L0 = bench.synth(m, n, B, 0, dev)
torch.manual_seed(1126)
net = dl.DLADMMNetScalar(m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0, E0=E0, L0=L0, layers=K)
net.requires_grad_(False)
tables = net._tables(dev); W = [w.detach() for w in net._weights()]
args = (net.VARIANT, X, net.A, W, net.Z0, net.E0, net.L0)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for e in ev:
    e.record()  # torch creates the hipEvent lazily: make the handles exist
res = {True: [], False: []}
for rep in range(12):
    for wp in (False, True):
        with torch.no_grad():
            r = ops.dladmm_forward(*args, keep_all=True, want_T=True, want_P=wp, loss_kind=1, kernel_events=ev, **tables)
        torch.cuda.synchronize()
        if rep >= 2: res[wp].append(ev[0].elapsed_time(ev[1]))
        del r
import statistics
print(json.dumps({"inference_ms": statistics.median(res[False]), "savep_ms": statistics.median(res[True])}))
