"""MinibatchSampler (src/main/scala/libs/MinibatchSampler.scala:1-60) and rank sharding.

SparkNet semantics: each round a worker draws a *random contiguous window* of
``num_sampled`` minibatches from its partition (start uniform in [0, total - num_sampled]),
and the image and label streams stay in lock-step whichever is consumed first.
"""
from __future__ import annotations

import random


class MinibatchSampler:
    def __init__(self, total_batches: int, num_sampled: int, seed: int | None = None):
        if num_sampled > total_batches:
            raise ValueError("cannot sample more minibatches than the partition holds")
        self.total = total_batches
        self.n = num_sampled
        self.rng = random.Random(seed)
        self.start = self.rng.randint(0, total_batches - num_sampled)
        self.image_pos = 0
        self.label_pos = 0

    def indices(self) -> list[int]:
        return list(range(self.start, self.start + self.n))

    def next_image_index(self) -> int:
        if self.image_pos >= self.n:
            raise StopIteration
        i = self.start + self.image_pos
        self.image_pos += 1
        return i

    def next_label_index(self) -> int:
        if self.label_pos >= self.n:
            raise StopIteration
        i = self.start + self.label_pos
        self.label_pos += 1
        return i

    def next_index(self) -> int:
        """Joint image+label draw (the usual path)."""
        i = self.next_image_index()
        self.label_pos = max(self.label_pos, self.image_pos)
        return i


class MinibatchStream:
    """Wrap per-partition minibatch lists with the sampler: next_image / next_label."""

    def __init__(self, image_batches, label_batches, num_sampled: int, seed: int | None = None):
        self.images, self.labels = image_batches, label_batches
        self.sampler = MinibatchSampler(len(image_batches), num_sampled, seed)

    def next_image_minibatch(self):
        return self.images[self.sampler.next_image_index()]

    def next_label_minibatch(self):
        return self.labels[self.sampler.next_label_index()]


def shard_range(n_items: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous deterministic shard (replaces Spark repartition/coalesce)."""
    per = n_items // world
    rem = n_items % world
    start = rank * per + min(rank, rem)
    return start, start + per + (1 if rank < rem else 0)
