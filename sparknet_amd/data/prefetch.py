"""Device input pipeline: pinned host uint8 minibatches -> side-stream H2D -> on-device
augment kernel -> the net's JavaData blobs.

Replaces SparkNet's JNA data callback (caffe/src/caffe/layers/java_data_layer.cpp:37-44,
src/main/scala/libs/Net.scala:194-233), which ran synchronously inside Forward and was
followed by an implicit synchronous H2D copy (caffe/src/caffe/syncedmem.cpp:61-69), and
Caffe's prefetch thread (base_data_layer.cpp:70-96).  Here:

* a host ring of pinned uint8 batches (raw planar CHW bytes, 4x smaller than float),
* ``hipMemcpyAsync`` of batch k+1 on a dedicated copy stream while step k computes,
* an event hand-off, then ONE augment launch (crop / mirror / mean / scale / NCHW->NHWC
  / uint8->bf16) on the compute stream writing straight into the data blob.
"""
from __future__ import annotations

import torch

from ..ops import _lib


class HostBatchSource:
    """Iterator protocol: ``next_batch() -> (uint8 [N,C,H,W] tensor, int32 [N] labels)``."""

    def next_batch(self):
        raise NotImplementedError


class SyntheticSource(HostBatchSource):
    """Synthetic uint8 images / labels of a fixed shape (the benchmark data): a small
    pool of random batches generated once and cycled, so the timed loop still moves a
    full minibatch over PCIe every step."""

    def __init__(self, batch, channels, height, width, classes=1000, pool=4, seed=0, pin=True):
        g = torch.Generator().manual_seed(seed)
        self.batches = []
        for _ in range(pool):
            x = torch.randint(0, 256, (batch, channels, height, width), dtype=torch.uint8, generator=g)
            y = torch.randint(0, classes, (batch,), dtype=torch.int32, generator=g)
            if pin and torch.cuda.is_available():
                x, y = x.pin_memory(), y.pin_memory()
            self.batches.append((x, y))
        self.i = 0

    def next_batch(self):
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b


class TensorSource(HostBatchSource):
    """Cycle over an in-memory uint8 dataset (e.g. CIFAR-10 from CifarLoader)."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, batch: int, sampler=None, pin=True):
        self.images, self.labels, self.batch = images, labels.int(), batch
        self.sampler = sampler
        self.pos = 0
        n = images.shape[0]
        self.nbatches = n // batch
        self.pin = pin and torch.cuda.is_available()

    def next_batch(self):
        if self.sampler is not None:
            idx = self.sampler.next_index()
        else:
            idx = self.pos % self.nbatches
            self.pos += 1
        sl = slice(idx * self.batch, (idx + 1) * self.batch)
        x, y = self.images[sl].contiguous(), self.labels[sl].contiguous()
        if self.pin:
            x, y = x.pin_memory(), y.pin_memory()
        return x, y


class WindowedSource(HostBatchSource):
    """SparkNet's per-round sampling: each round (``tau`` draws) uses a fresh random
    contiguous window of tau minibatches of this rank's shard (MinibatchSampler.scala:18-19)."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, batch: int, tau: int, seed: int = 0,
                 pin: bool = True):
        from .sampler import MinibatchSampler
        self._Sampler = MinibatchSampler
        self.images, self.labels, self.batch, self.tau = images, labels.int(), batch, tau
        self.nbatches = images.shape[0] // batch
        if self.nbatches < 1:
            raise ValueError("shard smaller than one minibatch")
        self.seed = seed
        self.round = 0
        self.sampler = None
        self.pin = pin and torch.cuda.is_available()

    def next_batch(self):
        if self.sampler is None or self.sampler.image_pos >= self.sampler.n:
            self.sampler = self._Sampler(self.nbatches, min(self.tau, self.nbatches), seed=self.seed * 7919 + self.round)
            self.round += 1
        idx = self.sampler.next_index()
        sl = slice(idx * self.batch, (idx + 1) * self.batch)
        x, y = self.images[sl].contiguous(), self.labels[sl].contiguous()
        if self.pin:
            x, y = x.pin_memory(), y.pin_memory()
        return x, y


class DeviceFeeder:
    """Double-buffered H2D + augment into a net's data/label blobs."""

    def __init__(self, source: HostBatchSource, data_blob, label_blob, *, crop: int | None = None,
                 mean=None, scale: float = 1.0, mirror: bool = False, train: bool = True,
                 rng_state: torch.Tensor | None = None, device="cuda", slots: int = 2, group: int = 2):
        self.source = source
        # group > 1: the H2D copies of `group` minibatches are issued together, one group
        # ahead, under ONE copy/compute fence pair (2*group slots), so the per-step
        # cross-stream synchronisation is amortised (docs/PERF_NOTES.md "Throughput phases").
        self.group = max(1, int(group))
        self.data_blob, self.label_blob = data_blob, label_blob
        self.device = torch.device(device)
        from .native import NativeLoader
        self.native = isinstance(source, NativeLoader)
        if self.native:
            x0 = y0 = None
            self.shape = tuple(source.shape)
        else:
            x0, y0 = source.batches[0] if isinstance(source, SyntheticSource) else source.next_batch()
            self.shape = tuple(x0.shape)
        N, C, H, W = self.shape
        self.crop = crop or H
        self.scale, self.mirror, self.train = scale, mirror, train
        self.mean_mode, self.mean = 0, None
        if mean is not None:
            m = torch.as_tensor(mean, dtype=torch.float32).to(self.device)
            self.mean_mode = 1 if m.numel() == C else 2
            self.mean = m.contiguous()
        self.rng_state = rng_state if rng_state is not None else torch.tensor([1, 0], dtype=torch.int64,
                                                                              device=self.device)
        self.copy_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        if self.copy_stream is None or getattr(source, "submitted", None) is not None:
            # Python ring sources recycle a host slot only when told about its copy event:
            # keep one copy per step (the native loader records its own per-copy events)
            self.group = 1
        if self.group > 1:
            slots = max(slots, 2 * self.group)
        self.slots = [(torch.empty(self.shape, dtype=torch.uint8, device=self.device),
                       torch.empty((N,), dtype=torch.int32, device=self.device)) for _ in range(slots)]
        self.events = [None] * slots
        self.fold = None  # (x2, plan, ConvSpec) when fused with the first conv's S2D fold
        self.k = 0
        self._pending = None
        if not isinstance(source, SyntheticSource) and not self.native:
            self._first = (x0, y0)
        else:
            self._first = None

    def prefetch(self) -> None:
        """Issue the H2D copy of the next host batch into the next slot (copy stream)."""
        if self.group > 1:
            self._prefetch_group()
            return
        if self.native:
            self._prefetch_native()
            return
        if self._first is not None:
            x, y = self._first
            self._first = None
        else:
            x, y = self.source.next_batch()
        slot = self.k % len(self.slots)
        dx, dy = self.slots[slot]
        if self.copy_stream is not None:
            # the slot is reused only after the compute stream consumed it
            self.copy_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.copy_stream):
                dx.copy_(x, non_blocking=True)
                dy.copy_(y, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.copy_stream)
            self.events[slot] = ev
        else:
            ev = None
            dx.copy_(x)
            dy.copy_(y)
        done = getattr(self.source, "submitted", None)  # ring sources recycle x after the copy
        if done is not None:
            done(x, ev)
        self._pending = slot
        self.k += 1

    def _next_host(self):
        if self._first is not None:
            x, y = self._first
            self._first = None
            return x, y
        return self.source.next_batch()

    def _issue_group(self, start: int) -> None:
        """Copy minibatches start .. start+group-1 into their slots behind one fence pair."""
        n = len(self.slots)
        cur = torch.cuda.current_stream(self.device)
        # slots (start + j) % n were last read by steps start-n+j, already submitted on cur
        self.copy_stream.wait_stream(cur)
        sent = []
        with torch.cuda.stream(self.copy_stream):
            for j in range(self.group):
                dx, dy = self.slots[(start + j) % n]
                if self.native:  # the C++ loader copies its next pinned slot on this stream
                    self.source.next_to_device(dx, dy, self.copy_stream)
                    continue
                x, y = self._next_host()
                dx.copy_(x, non_blocking=True)
                dy.copy_(y, non_blocking=True)
                sent.append(x)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        for j in range(self.group):
            # later slots of the group are ordered behind the first one's wait on the compute stream
            self.events[(start + j) % n] = ev if j == 0 else None
        done = getattr(self.source, "submitted", None)
        if done is not None:
            for x in sent:
                done(x, ev)

    def _prefetch_group(self) -> None:
        k, g = self.k, self.group
        if k == 0:
            self._issue_group(0)
        if k % g == 0:
            self._issue_group(k + g)  # one group ahead: `group` steps to hide `group` copies
        self._pending = k % len(self.slots)
        self.k += 1

    def _prefetch_native(self) -> None:
        """Native pipeline: the C++ loader issues the H2D copy of its next pinned slot."""
        slot = self.k % len(self.slots)
        dx, dy = self.slots[slot]
        if self.copy_stream is not None:
            self.copy_stream.wait_stream(torch.cuda.current_stream(self.device))
            self.source.next_to_device(dx, dy, self.copy_stream)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            self.events[slot] = ev
        else:
            _, x, y = self.source.next_host()
            dx.copy_(torch.from_numpy(x))
            dy.copy_(torch.from_numpy(y))
        self._pending = slot
        self.k += 1

    def stage(self) -> None:
        """Compute stream: wait for the slot, augment into the data blob, labels -> float."""
        if self._pending is None:
            self.prefetch()
        slot = self._pending
        self._pending = None
        if self.events[slot] is not None:
            torch.cuda.current_stream(self.device).wait_event(self.events[slot])
        src, lab = self.slots[slot]
        if self.device.type != "cuda":
            self._stage_cpu(src, lab)
            return
        from ..ops import hip
        ld = self.label_blob.data  # labels -> float inside the augment launch
        fused = ld.dtype == torch.float32 and ld.is_contiguous() and ld.numel() == lab.numel()
        labels, label_out = (lab, ld) if fused else (None, None)
        if self.fold is not None:
            x2, plan, spec = self.fold
            hip.augment_s2d(src, x2, self.crop, plan, spec, self.mean, self.mean_mode, self.scale, self.rng_state,
                            self.train, self.mirror, labels, label_out)
        else:
            hip.augment(src, self.data_blob.data, self.crop, self.mean, self.mean_mode, self.scale,
                        self.rng_state, self.train, self.mirror, labels=labels, label_out=label_out)
        if not fused:
            _lib.call("labels_to_float", lab, ld, lab.numel())

    def _stage_cpu(self, src, lab) -> None:
        """Reference (CPU) version of the augment kernel semantics."""
        x = src.float()
        N, C, H, W = x.shape
        if self.mean_mode == 1:
            x = x - self.mean.view(1, -1, 1, 1)
        elif self.mean_mode == 2:
            x = x - self.mean.view(1, C, H, W)
        c = self.crop
        out = torch.empty((N, C, c, c))
        if self.train and self.rng_state is not None:
            # the device kernels' Philox draw (ops.ref.augment_params): CPU and GPU feeders
            # fed the same batches at the same RNG counter produce the same crops
            from ..ops import ref
            st = self.rng_state.detach().cpu()
            params = ref.augment_params(N, int(st[0]), int(st[1]), H, W, c, c, bool(self.mirror))
        else:
            params = [((H - c) // 2, (W - c) // 2, False)] * N
        for n in range(N):
            ho, wo, mir = params[n]
            crop = x[n, :, ho:ho + c, wo:wo + c]
            out[n] = crop.flip(-1) if mir else crop
        self.data_blob.set_nchw(out * self.scale)
        self.label_blob.data.copy_(lab.float().reshape(self.label_blob.data.shape))

    def __call__(self, layer=None, tops=None) -> None:
        """JavaData-layer source hook (eager mode): stage + prefetch the next batch."""
        self.stage()
        self.prefetch()
