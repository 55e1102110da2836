"""Collectives over RCCL (torch.distributed backend "nccl" on ROCm) or gloo (CPU tests).

Replaces SparkNet's Spark-driver communication:

* K1 ``sc.broadcast(netWeights)`` + per-float JNA ``setWeights`` -> :meth:`broadcast_params`
  (once, at start: one broadcast of the flat fp32 buffer from rank 0);
* K2 ``workers.map(getWeights).reduce(WeightCollection.add)`` + ``scalarDivide(N)``
  (CifarApp.scala:133-134) -> :meth:`average_params`: all-reduce(SUM) of the flat fp32
  master buffer in large buckets, then ONE fused kernel that scales by 1/N and refreshes
  the bf16 compute shadow;
* K3 test-score reduce (CifarApp.scala:113-114) -> :meth:`allreduce_scores`;
* K4 partition-size collects -> :meth:`allgather_int`;
* K8 Caffe P2PSync gradient tree (caffe/src/caffe/parallel.cpp:287-380) ->
  :meth:`allreduce_grads` (synchronous-SGD mode).

Bucket size: xGMI is point-to-point (7 links x ~153 GB/s per MI355X); RCCL spreads one
large all-reduce over many channels, so buckets are large (default 256 MB) — they exist
only to bound transient memory and let the sync-SGD mode overlap with backward.
"""
from __future__ import annotations

import atexit
import datetime
import os
import sys
import threading

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 256 << 20
# weight averaging: 64 MB buckets (4 for CaffeNet's 244 MB) so the scale / shadow refresh of
# one bucket overlaps the next bucket's all-reduce; bench.py's comm_bench measures 256 / 64 / 16
AVERAGE_BUCKET_BYTES = 64 << 20
WATCHDOG_EXIT_CODE = 75



def _scale(flat: torch.Tensor, shadow, scale: float) -> None:
    """flat *= scale (and refresh its bf16 shadow): the HIP scale kernel on device
    buffers (one pass, vectorised, graph-capturable), plain in-place on host buffers."""
    if flat.is_cuda:
        from ..ops import hip
        hip.scale_shadow(flat, shadow, scale)
    else:
        flat.mul_(scale)
        if shadow is not None:
            shadow.copy_(flat)

class Watchdog:
    """Fail-fast rank monitor (the reference fails the whole Spark job on the
    first task failure, spark.task.maxFailures=1, src/main/scala/apps/CifarApp.scala:30).

    Every rank runs a daemon thread on its own client connection to the job's TCP store:
    it bumps its heartbeat counter every ``interval`` seconds and reads the peers'.  A
    peer whose counter has not moved for ``timeout`` seconds (process died: os._exit,
    segfault, OOM kill), a set ``abort`` key (a peer caught an exception and called
    :meth:`abort`) or a lost store connection ends this process with exit code 75
    within seconds — instead of blocking in the next all-reduce until the process-group
    timeout.  A rank that finishes normally marks itself done first (close / atexit), so
    peers never mistake a clean exit for a failure."""

    def __init__(self, rank: int, world: int, interval: float = 1.0, timeout: float | None = None,
                 prefix: str = "sn_watchdog"):
        self.rank, self.world, self.interval = rank, world, interval
        self.timeout = timeout if timeout is not None else float(os.environ.get("SN_WATCHDOG_TIMEOUT", "20"))
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ["MASTER_PORT"])
        base = dist.TCPStore(host, port, world, False, timeout=datetime.timedelta(seconds=30),
                             wait_for_workers=False)
        self.store = dist.PrefixStore(prefix, base)
        self._stop = threading.Event()
        self._done = False
        self.thread = threading.Thread(target=self._loop, name="sn-watchdog", daemon=True)
        self.thread.start()
        atexit.register(self.stop)

    def _fail(self, why: str) -> None:
        if self._stop.is_set():
            return
        print(f"[watchdog rank {self.rank}] {why}: exiting", file=sys.stderr, flush=True)
        os._exit(WATCHDOG_EXIT_CODE)

    def _loop(self) -> None:
        import time
        peers = [r for r in range(self.world) if r != self.rank]
        last = {r: (-1, time.monotonic()) for r in peers}
        while not self._stop.wait(self.interval):
            try:
                self.store.add(f"hb/{self.rank}", 1)
                if self.store.add("abort", 0) > 0:
                    self._fail("a peer requested an abort")
                now = time.monotonic()
                for r in peers:
                    v = self.store.add(f"hb/{r}", 0)
                    if v != last[r][0]:
                        last[r] = (v, now)
                    elif now - last[r][1] > self.timeout and self.store.add(f"done/{r}", 0) == 0:
                        self._fail(f"rank {r} stopped responding ({self.timeout:.0f} s without a heartbeat)")
            except Exception as e:  # store host gone: the job is failing
                if not self._stop.is_set():
                    self._fail(f"lost the job store ({type(e).__name__}: {e})")

    def abort(self) -> None:
        try:
            self.store.add("abort", 1)
        except Exception:
            pass

    def stop(self) -> None:
        if self._done:
            return
        self._done = True
        self._stop.set()
        try:
            self.store.add(f"done/{self.rank}", 1)
        except Exception:
            pass
        self.thread.join(timeout=5)


class Comm:
    def __init__(self, backend: str | None = None, device=None, timeout_s: float = 1800.0,
                 bucket_bytes: int = DEFAULT_BUCKET_BYTES, watchdog: bool = False):
        self.bucket_bytes = bucket_bytes
        self.average_bucket_bytes = AVERAGE_BUCKET_BYTES
        self.watchdog = None
        # SN_COMM_FORCE=1: set up the process group and run every collective even at world 1
        # (one GPU under torch.distributed.run --nproc-per-node 1): an RCCL rehearsal of the
        # scaling path's exact call pattern on a single-GPU box (scripts/gpu_r5ap.sh)
        force = os.environ.get("SN_COMM_FORCE", "0") == "1" and "MASTER_ADDR" in os.environ
        if dist.is_available() and dist.is_initialized():
            self.owns = False
        elif int(os.environ.get("WORLD_SIZE", "1")) > 1 or force:
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            kw = {}
            if backend == "nccl" and device is not None:
                kw["device_id"] = torch.device(device)
            dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
            self.owns = True
        else:
            self.owns = False
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.backend = dist.get_backend() if dist.is_initialized() else None
        # collectives run when there is more than one rank, or when forced at world 1
        self.active = self.world_size > 1 or (force and dist.is_initialized())
        if watchdog and self.world_size > 1 and "MASTER_PORT" in os.environ:
            self.watchdog = Watchdog(self.rank, self.world_size)

    # -- helpers ------------------------------------------------------------------------
    def _buckets(self, flat: torch.Tensor):
        n = flat.numel()
        per = max(1, self.bucket_bytes // flat.element_size())
        for s in range(0, n, per):
            yield flat[s:s + per]

    def barrier(self) -> None:
        if self.active:
            dist.barrier()

    # -- parameter sync -------------------------------------------------------------------
    def broadcast_params(self, net, src: int = 0) -> None:
        if not self.active:
            return
        for b in self._buckets(net.flat_data):
            dist.broadcast(b, src)
        net.sync_compute()

    def allreduce_sum(self, flat: torch.Tensor, async_op: bool = False):
        works = [dist.all_reduce(b, op=dist.ReduceOp.SUM, async_op=async_op) for b in self._buckets(flat)]
        return works if async_op else None

    def bucket_ranges(self, n: int, bucket_bytes: int | None = None, elem: int = 4):
        per = max(1, (bucket_bytes or self.bucket_bytes) // elem)
        return [(s, min(n, s + per)) for s in range(0, n, per)]

    def average_params(self, net, bucket_bytes: int | None = None) -> list[float]:
        """Model averaging: every rank ends with the exact same mean weights.

        The flat fp32 master buffer is all-reduced in buckets issued together as async
        collectives; each bucket's 1/N scale + bf16 shadow refresh (``hip.scale_shadow``)
        is enqueued as soon as THAT bucket's all-reduce is waited for, so on RCCL the
        scaling of bucket i runs on the compute stream while bucket i+1 is still on the
        wire.  Returns the host-side issue time per bucket (ms; GPU timing is the
        caller's, e.g. bench.py's events)."""
        if not self.active:
            return []
        import time
        flat = net.flat_data
        scale = 1.0 / self.world_size
        cuda = flat.is_cuda
        shadow = net.flat_compute if cuda and net.flat_compute is not net.flat_data else None
        ranges = self.bucket_ranges(flat.numel(), bucket_bytes or self.average_bucket_bytes)
        works, t = [], []
        for s, e in ranges:
            t0 = time.perf_counter()
            works.append(self.allreduce_sum(flat[s:e], async_op=True) or ())
            t.append(1e3 * (time.perf_counter() - t0))
        for (s, e), ws in zip(ranges, works):
            for w in ws:
                w.wait()
            _scale(flat[s:e], shadow[s:e] if shadow is not None else None, scale)
        if not cuda:
            net.sync_compute()
        return t

    def allreduce_grads(self, net, average: bool = True) -> None:
        """Synchronous data-parallel SGD: sum (or average) the flat gradient buffer."""
        if not self.active:
            return
        self.allreduce_sum(net.flat_diff)
        if average:
            _scale(net.flat_diff, None, 1.0 / self.world_size)

    def allreduce_scores(self, scores: list[float], device=None) -> list[float]:
        if not self.active:
            return list(scores)
        t = torch.tensor(list(scores), dtype=torch.float64 if device is None else torch.float32,
                         device=device or "cpu")
        if device is None and dist.get_backend() == "nccl":
            t = t.float().cuda()
        dist.all_reduce(t)
        return t.cpu().tolist()

    def allgather_int(self, v: int) -> list[int]:
        if not self.active:
            return [v]
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([v], dtype=torch.int64, device=dev)
        out = [torch.zeros_like(t) for _ in range(self.world_size)]
        dist.all_gather(out, t)
        return [int(x.item()) for x in out]

    def allgather_float(self, v: float) -> list[float]:
        if not self.active:
            return [v]
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        out = [torch.zeros_like(t) for _ in range(self.world_size)]
        dist.all_gather(out, t)
        return [float(x.item()) for x in out]

    def max_over_ranks(self, v: float) -> float:
        if not self.active:
            return v
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([v], dtype=torch.float64 if dev == "cpu" else torch.float32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def abort(self) -> None:
        """Tell every peer to exit now (called when this rank hits an error)."""
        if self.watchdog is not None:
            self.watchdog.abort()

    def close(self) -> None:
        if self.watchdog is not None:
            # every rank marks itself done before any rank (possibly the store host) exits
            self.watchdog.stop()
            self.barrier()
            self.watchdog = None
        if self.owns and dist.is_initialized():
            dist.destroy_process_group()


def grad_buckets(net, bucket_bytes: int):
    """Plan the overlapped gradient all-reduce: ({layer index: [(start, end), ...]}, late
    ranges).  A parameter's gradient is final after the backward of the LAST layer (in
    backward order) that writes it; parameters are packed in backward order into
    contiguous flat ranges of >= ``bucket_bytes`` that are launched from the backward
    hook of the layer completing them.  Gradients that backward does not write (frozen /
    pruned layers, zeroed by Net.finish_param_diffs) form the late ranges."""
    from ..core.net import PARAM_ALIGN
    users, late = {}, set()
    for li, layer in enumerate(net.layers):
        for i, p in enumerate(layer.params):
            users[p.offset] = min(users.get(p.offset, li), li)
            if not net.layer_need_backward[li] or not layer.param_grads_needed(i):
                late.add(p.offset)
    seg = {p.offset: -(-p.count // PARAM_ALIGN) * PARAM_ALIGN for p in net.learnable_params}
    order = sorted((o for o in seg if o in users and o not in late), key=lambda o: (-users[o], -o))
    plan, cur, cur_bytes = {}, [], 0

    def close(at_layer):
        nonlocal cur, cur_bytes
        if not cur:
            return
        lo, hi = min(cur), max(o + seg[o] for o in cur)
        ranges = [(lo, hi)] if hi - lo == sum(seg[o] for o in cur) else [(o, o + seg[o]) for o in sorted(cur)]
        plan.setdefault(at_layer, []).extend(ranges)
        cur, cur_bytes = [], 0

    for k, o in enumerate(order):
        cur.append(o)
        cur_bytes += seg[o] * 4
        nxt = order[k + 1] if k + 1 < len(order) else None
        if cur_bytes >= bucket_bytes or nxt is None or (users[nxt] != users[o] and cur_bytes >= bucket_bytes):
            close(users[o])
    late_ranges = [(o, o + seg[o]) for o in sorted(seg) if o in late or o not in users]
    return plan, late_ranges


class SyncSGDCallback:
    """Solver callback for synchronous gradient all-reduce (Caffe P2PSync semantics:
    N ranks x batch B == 1 rank x batch N*B, test_gradient_based_solver.cpp:455-490).

    With ``overlap`` (default) the flat gradient buffer is all-reduced in buckets
    launched asynchronously from the backward pass as soon as each bucket's gradients
    are final (fc8/fc7/fc6 first in CaffeNet), so the collective runs under the remaining
    backward GEMMs; ``on_gradients_ready`` waits for them, reduces the rest and scales by
    1/N."""

    def __init__(self, comm: Comm, net, overlap: bool = True, bucket_bytes: int = 32 << 20):
        self.comm, self.net = comm, net
        self.works = []
        self.plan = None
        if overlap and comm.active:
            self.plan, self.late = grad_buckets(net, bucket_bytes)
            net.backward_hooks.append(self._hook)

    def on_start(self):
        self.works = []

    def _hook(self, li: int) -> None:
        for s, e in self.plan.get(li, ()):
            self.works.append(dist.all_reduce(self.net.flat_diff[s:e], op=dist.ReduceOp.SUM, async_op=True))

    def on_gradients_ready(self):
        if self.plan is None:
            self.comm.allreduce_grads(self.net, average=True)
            return
        for w in self.works:
            w.wait()
        self.works = []
        for s, e in self.late:
            dist.all_reduce(self.net.flat_diff[s:e], op=dist.ReduceOp.SUM)
        _scale(self.net.flat_diff, None, 1.0 / self.comm.world_size)
