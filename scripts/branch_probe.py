"""Reproduce the multi-stream capture of a tiny GoogLeNet with a native backtrace."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BT = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libsegv_bt.so"))
import torch  # noqa: E402
from sparknet_amd import models, proto  # noqa: E402
from sparknet_amd.core.net import Net  # noqa: E402
from sparknet_amd.engine import BranchStreams, fuse_relu  # noqa: E402

nstreams = int(sys.argv[1]) if len(sys.argv) > 1 else 4
limit = int(sys.argv[2]) if len(sys.argv) > 2 else 10**9
n = models.googlenet(train_batch=4, test_batch=4, crop=67, classes=7, aux=True)
for l in n.layer:
    if l.type == "Dropout":
        l.dropout_param.dropout_ratio = 0.0
    if l.name in ("pool5/7x7_s1", "loss1/ave_pool", "loss2/ave_pool"):
        for f in ("kernel_h", "kernel_w", "stride_h", "stride_w", "kernel_size", "stride"):
            l.pooling_param.ClearField(f)
        l.pooling_param.global_pooling = True
net = Net(n, phase=proto.TRAIN, seed=3, device="cuda")
fuse_relu(net)
net.blob_by_name("data").set_nchw(torch.randn(4, 3, 67, 67) * 20)
net.blob_by_name("label").set_nchw(torch.tensor([[1.0], [5.0], [0.0], [6.0]]))
bs = BranchStreams(net, nstreams, star=os.environ.get('SN_STAR') == '1')
print('streams used', bs.streams_used(), bs.streams_used(True), flush=True)
for plan in (bs.fwd_plan, bs.bwd_plan):  # nodes past `limit` go to stream 0 with full waits
    pass
net.clear_param_diffs()
bs.forward_backward()
torch.cuda.synchronize()
print("eager ok", flush=True)
BT.sn_install_segv_bt()
import faulthandler; faulthandler.disable()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    bs.forward_backward()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print("side-stream eager ok", flush=True)
g = torch.cuda.CUDAGraph()
which = sys.argv[3] if len(sys.argv) > 3 else "both"
import traceback  # noqa: E402
cs = torch.cuda.Stream()
cs.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(cs):
    g.capture_begin()
    try:
        if which == "fwd":
            bs.forward()
        else:
            bs.forward_backward()
        print("body ok", flush=True)
    except BaseException:
        traceback.print_exc()
        sys.stdout.flush(); sys.stderr.flush()
        os._exit(3)
    g.capture_end()
torch.cuda.current_stream().wait_stream(cs)
print("capture ok", flush=True)
g.replay()
torch.cuda.synchronize()
print("replay ok", flush=True)
