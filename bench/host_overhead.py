import sys, time, torch, os
sys.path.insert(0, os.getcwd())
from dalgo.data.datasets import synthetic_logistic
from dalgo.models.localsgd import ParallelSGD, SGDConfig
from dalgo.parallel import runtime
from dalgo.parallel.sharding import make_layout
rt = runtime.init(device="cuda")
rows = int(sys.argv[1])
layout = make_layout(rows, 1, 1, 0, spark_compatible=False)
data = synthetic_logistic(rows, 1024, row_range=(0, rows), device=rt.device, dtype=torch.bfloat16)
m = ParallelSGD(SGDConfig(algo="ssgd", n_workers=1, frac=0.1, eval_every=0, n_iterations=10), data, layout, rt)
for _ in range(20): m.step()
torch.cuda.synchronize()
n = 300
t0 = time.perf_counter()
for _ in range(n): m.step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"rows={rows} host {1e6*(t1-t0)/n:.1f} us/step, wall {1e6*(t2-t0)/n:.1f} us/step")
from dalgo.ops import lr as L
X, y, W, seg = data.X_train, data.y_train, m.w, m.seg
t0 = time.perf_counter()
for i in range(n): L.lr_grad(X, y, W, seg, D=1024, frac=0.1, step=i, G=m.G, C=m.C, g_is_zero=True)
t1 = time.perf_counter(); torch.cuda.synchronize()
print(f"lr_grad wrapper host {1e6*(t1-t0)/n:.1f} us/call")
