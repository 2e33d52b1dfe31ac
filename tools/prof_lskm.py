import importlib, sys, os, time, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import bench
dl = importlib.import_module("d-ladmm_amd")
dev = torch.device("cuda", 0)
A, X, Z0, E0, L0 = bench.synth(250, 500, 1000, 0, dev)
net = dl.DLADMMNetLSKM(m=250, n=0, d=500, batch_size=1000, A=A, Z0=Z0, E0=E0, L0=L0, layers=20,
                       alpha=0.01, mu_k_method="EMA", mu_k_param=0.5).cuda()
for _ in range(3): net(X, True, True, False)
torch.cuda.synchronize()
t0 = time.perf_counter(); net(X, True, True, False); t1 = time.perf_counter()
torch.cuda.synchronize(); t2 = time.perf_counter()
print("host issue ms", (t1 - t0) * 1e3, "wall ms", (t2 - t0) * 1e3)
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as p:
    net(X, True, True, False); torch.cuda.synchronize()
print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))
print(p.key_averages().table(sort_by="self_cuda_time_total", row_limit=15))
