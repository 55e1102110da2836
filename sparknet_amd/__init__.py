"""sparknet_amd — MI355X-native parallel-SGD CNN training engine (SparkNet's capabilities,
Caffe's NetParameter / .caffemodel formats)."""
import os

# Multi-process GPU work (RCCL, CUDA-tensor sharing) needs the dmabuf IPC mode, the only one
# the host driver supports; the HSA runtime reads this when HIP initialises, so set it before
# any entry point (bench.py, apps, torchrun workers, the C ABI's embedded interpreter) can
# touch the GPU.  An explicit setting in the environment wins.
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
