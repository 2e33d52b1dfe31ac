"""Per-wave cycle shares of a fused forward kernel from its diagnostic stamp build.

    python tools/x3_ablate.py X3_STAMP=1                                    # split-f16 (CPU)
    DLADMM_LIB=d-ladmm_amd/lib/abl/libdladmm_hip_x3ablX3_STAMP1.so python tools/x3_stamp.py
    python tools/ablate.py stamp=-DDLADMM_STAMP=1                           # fp32 kernel
    DLADMM_LIB=d-ladmm_amd/lib/abl/stamp/libdladmm_hip.so python tools/x3_stamp.py f32

Runs the headline workload (V4, m=256, n=512, K=15, B=65536, all layers written) a few times
and prints the mean over waves of: total cycles, G1 passes, G2 passes, between passes, ring
barrier vmcnt waits and s_barrier waits.  Read the shares, not the absolute time: each stamp
drains the wave's LDS reads.
"""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    dev = torch.device("cuda", 0)
    B, m, n, K = 65536, 256, 512, 15
    dbg = torch.zeros(B // 16 * 8, dtype=torch.int64, device=dev)
    os.environ["DLADMM_DBG_PTR"] = str(dbg.data_ptr())
    import bench
    dl = importlib.import_module("d-ladmm_amd")
    A, X, Z0, E0, L0 = bench.synth(m, n, B, 0, dev)
    net = dl.DLADMMNetScalar(m=m, n=0, d=n, batch_size=B, A=A, Z0=Z0, E0=E0, L0=L0, layers=K)
    net.precision = sys.argv[1] if len(sys.argv) > 1 else "f32_split"
    net.requires_grad_(False)
    with torch.no_grad():
        for _ in range(3):
            r = net.run(X, keep_all=True, loss_kind=dl._lib.LOSS_L1L1)
            del r
    torch.cuda.synchronize()
    v = dbg.view(-1, 8).double().mean(0).tolist()
    names = ["total", "g1_passes", "g2_passes", "between", "ring_vmcnt", "ring_barrier"]
    tot = v[0]
    for i, nm in enumerate(names):
        print(f"{nm:14s} {v[i]:14.0f} cycles  {v[i] / tot:6.3f}")
    # spread over waves of the total (imbalance)
    t = dbg.view(-1, 8)[:, 0].double()
    print(f"total min/max over waves: {t.min().item():.0f} / {t.max().item():.0f}")


if __name__ == "__main__":
    main()
