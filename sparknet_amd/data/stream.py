"""Bounded-memory ImageNet ingest: compressed records streamed from this rank's shards,
decoded by a worker pool into a ring of pinned minibatch buffers.

The reference keeps each partition's minibatches JPEG-compressed in the RDD and
decompresses one minibatch at a time (src/main/scala/apps/ImageNetApp.scala:60-62,
src/main/scala/loaders/ScaleAndConvert.scala:45-70); the mean image is computed from
those minibatches (ImageNetApp.scala:76, ComputeMean.scala).  Here:

* a reader thread walks the rank's tar shards (local or S3, ``ImageNetLoader._members``)
  record by record — with at least ``world`` shard files each rank reads only its own
  files (one partition per file, as the reference), otherwise records are dealt
  round-robin — optionally through a shuffle buffer of COMPRESSED records;
* ``workers`` threads decode + resize (PIL releases the GIL in its codecs) one
  minibatch at a time into one of ``slots`` pinned uint8 buffers;
* the device feeder's H2D copy of a slot is tracked with its CUDA event
  (``submitted``); the slot is rewritten only after that copy has completed.

Host RAM is ``slots * batch * C * H * W`` bytes plus the shuffle buffer: independent of
the shard size (the round-1 path decoded the whole shard, ~31 GB per rank at 8 ranks).
``epochs=None`` cycles forever (training); ``epochs=1`` ends the stream after one pass
(mean image, evaluation) — ``next_batch`` then raises StopIteration.
"""
from __future__ import annotations

import queue
import random
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from .loaders import ImageNetLoader, decode_resize
from .prefetch import HostBatchSource

_END = object()


class StreamingJpegSource(HostBatchSource):
    def __init__(self, loader: ImageNetLoader, batch: int, shard: tuple[int, int] = (0, 1), *, slots: int = 4,
                 workers: int = 8, shuffle_buffer: int = 0, seed: int = 0, epochs: int | None = None,
                 max_images: int = 0, pin: bool = True):
        if slots < 2:
            raise ValueError("need at least 2 ring slots")
        self.loader, self.batch, self.shard = loader, batch, shard
        self.epochs, self.max_images = epochs, max_images
        self.shuffle_buffer, self.seed = shuffle_buffer, seed
        H, W = loader.size
        self.shape = (batch, 3, H, W)
        pin = pin and torch.cuda.is_available()
        self.ring = []
        for _ in range(slots):
            x = torch.empty(self.shape, dtype=torch.uint8)
            y = torch.empty((batch,), dtype=torch.int32)
            self.ring.append((x.pin_memory(), y.pin_memory()) if pin else (x, y))
        self.events: list = [None] * slots
        self.free: queue.Queue = queue.Queue()
        for i in range(slots):
            self.free.put(i)
        self.ready: queue.Queue = queue.Queue()
        self.pool = ThreadPoolExecutor(max(1, workers), thread_name_prefix="sn-jpeg")
        self._stop = threading.Event()
        self._error: BaseException | None = None
        self._out: dict[int, int] = {}  # id(x) of a handed-out slot -> slot index
        self.batches_out = 0
        self.images_skipped = 0
        self.thread = threading.Thread(target=self._run, name="sn-jpeg-batcher", daemon=True)
        self.thread.start()

    # -- reader: this rank's compressed records, epoch after epoch ----------------------
    def _records(self):
        rank, world = self.shard
        files = self.loader.files()
        by_file = len(files) >= world > 1
        mine = files[rank::world] if by_file else files
        rng = random.Random(self.seed * 1_000_003 + rank)
        epoch = 0
        while self.epochs is None or epoch < self.epochs:
            buf = []
            n = 0
            for i, (name, data) in enumerate(self.loader._members(mine)):
                if self._stop.is_set():
                    return
                if not by_file and i % world != rank:
                    continue
                if self.max_images and n >= self.max_images:
                    break
                n += 1
                rec = (data, self.loader.labels.get(name, 0))
                if self.shuffle_buffer > 1:
                    if len(buf) < self.shuffle_buffer:
                        buf.append(rec)
                        continue
                    j = rng.randrange(len(buf))
                    buf[j], rec = rec, buf[j]
                yield rec
            rng.shuffle(buf)
            yield from buf
            epoch += 1
            if n == 0:
                return  # an empty shard would spin forever

    def _decode(self, rec):
        return decode_resize(rec[0], self.loader.size), rec[1]

    # -- batcher: decode one minibatch in parallel, write it into a free ring slot ---------
    def _run(self):
        try:
            recs = self._records()
            pending = []
            done = False
            while not self._stop.is_set() and not done:
                while len(pending) < self.batch:
                    need = self.batch - len(pending)
                    chunk = []
                    for rec in recs:
                        chunk.append(rec)
                        if len(chunk) == need:
                            break
                    if not chunk:
                        done = True  # end of the stream: the partial batch is dropped
                        break
                    for img, lab in self.pool.map(self._decode, chunk):
                        if img is None:
                            self.images_skipped += 1  # undecodable: skipped, as the reference
                        else:
                            pending.append((img, lab))
                if done or self._stop.is_set():
                    break
                slot = self.free.get()
                if slot is None:
                    break
                ev = self.events[slot]
                if ev is not None:
                    ev.synchronize()  # the previous H2D copy out of this slot has landed
                    self.events[slot] = None
                x, y = self.ring[slot]
                xn = x.numpy()
                for i, (img, lab) in enumerate(pending[:self.batch]):
                    xn[i] = img
                y.copy_(torch.tensor([lab for _, lab in pending[:self.batch]], dtype=torch.int32))
                pending = pending[self.batch:]
                self.ready.put(slot)
        except BaseException as e:  # surfaced to the consumer
            self._error = e
        self.ready.put(_END)

    # -- consumer ----------------------------------------------------------------------
    def next_batch(self):
        slot = self.ready.get()
        if slot is _END:
            self.ready.put(_END)
            if self._error is not None:
                raise RuntimeError("streaming JPEG source failed") from self._error
            raise StopIteration
        x, y = self.ring[slot]
        self._out[id(x)] = slot
        self.batches_out += 1
        return x, y

    def submitted(self, x: torch.Tensor, event) -> None:
        """The feeder has issued the copy out of ``x`` (CUDA ``event`` marks its end, None
        for a synchronous copy): the slot may be refilled once the copy has completed."""
        slot = self._out.pop(id(x), None)
        if slot is None:
            return
        self.events[slot] = event
        self.free.put(slot)

    def __iter__(self):
        while True:
            try:
                x, y = self.next_batch()
            except StopIteration:
                return
            yield x, y
            self.submitted(x, None)

    def host_bytes(self) -> int:
        return sum(x.numel() + 4 * y.numel() for x, y in self.ring)

    def close(self) -> None:
        self._stop.set()
        self.free.put(None)
        self.thread.join(timeout=10)
        self.pool.shutdown(wait=False, cancel_futures=True)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def streamed_mean(loader: ImageNetLoader, batch: int, shard=(0, 1), comm=None, max_images: int = 0,
                  workers: int = 8) -> np.ndarray:
    """Mean image of this rank's shard (one decoding pass, bounded memory), all-reduced
    over ranks: ComputeMean over the minibatches (ImageNetApp.scala:76)."""
    from .loaders import compute_mean
    src = StreamingJpegSource(loader, batch, shard, slots=2, workers=workers, epochs=1, max_images=max_images,
                              pin=False)
    try:
        return compute_mean((x for x, _ in src), comm)
    finally:
        src.close()
