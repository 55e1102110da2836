"""cifar10_quick on the synthetic pattern set of tests/test_training_gpu.py, trained by the
fp32 CPU engine (the numerics oracle): does the loss spike without any GPU kernel?

python scripts/cifar_quick_cpu_traj.py [seed] [steps] [lr]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

from sparknet_amd import models  # noqa: E402
from sparknet_amd.core.solver import Solver  # noqa: E402
from test_training_gpu import _patterns  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 5
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
torch.set_num_threads(8)
x, y = _patterns(2000)
sp = models.solver_for("cifar10_quick", train_batch=100, test_batch=100)
if len(sys.argv) > 3:
    sp.base_lr = float(sys.argv[3])
solver = Solver(sp, device=torch.device("cpu"), seed=seed, build_test_nets=False)
net = solver.net
m = torch.tensor([125.0, 123.0, 114.0]).view(1, 3, 1, 1)
losses = []
for it in range(steps):
    b = it % 20
    net.blob_by_name("data").set_nchw(x[b * 100:(b + 1) * 100].float() - m)
    net.blob_by_name("label").set_nchw(y[b * 100:(b + 1) * 100].float().view(-1, 1))
    losses.append(float(solver.iteration()))
    solver.iter += 1
    if it % 25 == 0:
        print(it, f"{losses[-1]:.4f}", flush=True)
print("cpu fp32 seed", seed, "final", f"{losses[-1]:.4f}", "max after 100", f"{max(losses[100:] or [0]):.4f}")
