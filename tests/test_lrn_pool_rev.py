"""Host-side eligibility of the LRN -> max-pool backward fusion (engine.fuse_lrn_pool_backward,
csrc/kernels/pool_lrn.hip: pool_lrn_bwd_rev); the kernel and net-level tests are in
tests/test_pool_lrn_gpu.py.  Reference: caffe/src/caffe/layers/lrn_layer.cu:121-177,
pooling_layer.cu:217-260 (the two backwards the fused launch replaces)."""
from sparknet_amd.ops.spec import PoolSpec


def test_lrn_pool_rev_eligibility():
    from sparknet_amd.ops import hip
    ok = PoolSpec(2, 27, 27, 256, 3, 3, 2, 2, 0, 0)
    assert hip.pool_lrn_rev_eligible(ok, 5, False)
    assert not hip.pool_lrn_rev_eligible(ok, 5, True)            # within-channel LRN
    assert not hip.pool_lrn_rev_eligible(ok, 4, False)           # even size
    assert not hip.pool_lrn_rev_eligible(PoolSpec(2, 27, 27, 20, 3, 3, 2, 2, 0, 0), 5, False)  # C % 8
    assert not hip.pool_lrn_rev_eligible(PoolSpec(2, 27, 27, 256, 2, 2, 2, 2, 0, 0), 5, False)
    assert not hip.pool_lrn_rev_eligible(PoolSpec(2, 27, 27, 256, 3, 3, 2, 2, 0, 0, 1), 5, False)  # AVE


def test_fuse_pass_is_gpu_only():
    import torch
    from sparknet_amd import engine, models
    from sparknet_amd.core.solver import Solver
    sp = models.zoo.solver_for("alexnet", train_batch=2, test_batch=2, crop=67, classes=10)
    net = Solver(sp, device=torch.device("cpu"), seed=1, build_test_nets=False).net
    assert engine.fuse_lrn_pool_backward(net) == 0
    assert all(getattr(l, "bwd_lrn", None) is None for l in net.layers)
