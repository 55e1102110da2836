"""Native minibatch pipeline (csrc/runtime/loader.cpp) — record decoding, the three
samplers, rank sharding and thread-count independence, on the CPU (unpinned ring).
Reference analogue: MinibatchSamplerSpec (src/test/scala/libs/MinibatchSamplerSpec.scala)
and CifarLoader (src/main/scala/loaders/CifarLoader.scala)."""
import os

import numpy as np
import pytest
import torch

from sparknet_amd.data import native
from sparknet_amd.data.loaders import CIFAR_RECORD, write_synthetic_cifar


@pytest.fixture(scope="module")
def cifar_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("cifar")
    write_synthetic_cifar(str(d), n_train=500, n_test=50, seed=3)
    return d


def _files(d):
    return [os.path.join(d, f"data_batch_{i}.bin") for i in range(1, 6)]


def _records(d):
    recs = np.concatenate([np.fromfile(f, dtype=np.uint8).reshape(-1, CIFAR_RECORD) for f in _files(d)])
    return recs[:, 1:].reshape(-1, 3, 32, 32), recs[:, 0].astype(np.int32)


def test_sequential_decodes_cifar_records(cifar_dir):
    imgs, labs = _records(cifar_dir)
    with native.NativeLoader.cifar10(_files(cifar_dir), 32, sampler=native.SAMPLER_SEQUENTIAL, pinned=False,
                                     threads=3) as L:
        for b in range(20):  # wraps around the 500-record shard
            seq, x, y = L.next_host()
            assert seq == b
            idx = [(b * 32 + i) % 500 for i in range(32)]
            assert np.array_equal(x, imgs[idx]) and np.array_equal(y, labs[idx])


def test_shuffle_is_a_permutation_per_epoch(cifar_dir):
    with native.NativeLoader.cifar10(_files(cifar_dir), 50, sampler=native.SAMPLER_SHUFFLE, seed=7,
                                     pinned=False) as L:
        assert L.stats()["batches_per_epoch"] == 10
        e0 = sum((L.batch_indices(b) for b in range(10)), [])
        e1 = sum((L.batch_indices(b) for b in range(10, 20)), [])
        assert sorted(e0) == list(range(500)) and sorted(e1) == list(range(500))
        assert e0 != e1 and e0 != list(range(500))


def test_window_sampler_matches_sparknet_semantics(cifar_dir):
    """Each round of tau batches is a contiguous window of minibatches starting uniformly
    in [0, P - tau] (MinibatchSampler.scala:18-34)."""
    tau, B = 3, 25  # P = 20 minibatches in the shard
    with native.NativeLoader.cifar10(_files(cifar_dir), B, sampler=native.SAMPLER_WINDOW, tau=tau, seed=1,
                                     pinned=False) as L:
        starts = set()
        for r in range(30):
            mb = []
            for j in range(tau):
                ix = L.batch_indices(r * tau + j)
                assert ix == list(range(ix[0], ix[0] + B)) and ix[0] % B == 0
                mb.append(ix[0] // B)
            assert mb == list(range(mb[0], mb[0] + tau)) and 0 <= mb[0] <= 20 - tau
            starts.add(mb[0])
        assert len(starts) > 5  # the window start is random per round


def test_rank_shards_are_disjoint_and_cover(cifar_dir):
    seen = []
    for rank in range(3):
        with native.NativeLoader.cifar10(_files(cifar_dir), 10, sampler=native.SAMPLER_SEQUENTIAL, rank=rank,
                                         world=3, pinned=False) as L:
            n = L.stats()["shard_samples"]
            _, x, _ = L.next_host()
            seen.append(n)
    assert sum(seen) == 500 and max(seen) - min(seen) <= 1


def test_memory_source_and_thread_independence():
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (300, 3, 8, 8), dtype=np.uint8)
    labs = rng.integers(0, 10, 300).astype(np.int32)
    outs = []
    for threads in (1, 4):
        with native.NativeLoader((3, 8, 8), 16, source=native.SOURCE_MEMORY, images=imgs, labels=labs,
                                 sampler=native.SAMPLER_SHUFFLE, seed=5, threads=threads, slots=3,
                                 pinned=False) as L:
            got = [L.next_host() for _ in range(25)]
            for seq, x, y in got:
                ix = L.batch_indices(seq)
                assert np.array_equal(x, imgs[ix]) and np.array_equal(y, labs[ix])
            outs.append(np.concatenate([g[1] for g in got]))
    assert np.array_equal(outs[0], outs[1])


def test_synthetic_source_is_deterministic():
    a = native.NativeLoader((3, 16, 16), 8, seed=9, pinned=False, classes=10)
    b = native.NativeLoader((3, 16, 16), 8, seed=9, pinned=False, classes=10, threads=3)
    for _ in range(5):
        _, xa, ya = a.next_host()
        _, xb, yb = b.next_host()
        assert np.array_equal(xa, xb) and np.array_equal(ya, yb)
        assert ya.min() >= 0 and ya.max() < 10
    a.close()
    b.close()


def test_bad_config_raises():
    with pytest.raises(RuntimeError):
        native.NativeLoader((3, 8, 8), 16, source=native.SOURCE_FILES, paths=["/nonexistent/x.bin"],
                            record=(0, 193, 0, 1, 1), pinned=False)


@pytest.mark.gpu
def test_next_to_device(gpu, cifar_dir):
    imgs, labs = _records(cifar_dir)
    dx = torch.empty((32, 3, 32, 32), dtype=torch.uint8, device=gpu)
    dy = torch.empty((32,), dtype=torch.int32, device=gpu)
    st = torch.cuda.Stream(gpu)
    with native.NativeLoader.cifar10(_files(cifar_dir), 32, sampler=native.SAMPLER_SEQUENTIAL, threads=2) as L:
        assert L.pinned
        for b in range(12):
            seq = L.next_to_device(dx, dy, st)
            st.synchronize()
            idx = [(seq * 32 + i) % 500 for i in range(32)]
            assert np.array_equal(dx.cpu().numpy(), imgs[idx]) and np.array_equal(dy.cpu().numpy(), labs[idx])


@pytest.mark.gpu
def test_grouped_feeder_over_native_loader(gpu, cifar_dir):
    """DeviceFeeder(group=3) over the C++ loader: three next_to_device copies per fence
    pair, staged labels follow the sequential sampler step for step."""
    from sparknet_amd import models
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.data.prefetch import DeviceFeeder
    _, labs = _records(cifar_dir)
    solver = Solver(models.solver_for("cifar10_quick", train_batch=10, test_batch=10), device=gpu, seed=5,
                    build_test_nets=False)
    net = solver.net
    with native.NativeLoader.cifar10(_files(cifar_dir), 10, sampler=native.SAMPLER_SEQUENTIAL, threads=2) as L:
        f = DeviceFeeder(L, net.blob_by_name("data"), net.blob_by_name("label"), crop=32, mirror=False,
                         train=False, rng_state=net.ctx.rng_state, device=gpu, group=3)
        assert f.group == 3 and len(f.slots) == 6
        for step in range(13):
            f.stage()
            f.prefetch()
            got = net.blob_by_name("label").data.float().cpu().flatten().numpy()
            want = labs[[(step * 10 + i) % 500 for i in range(10)]].astype(np.float32)
            assert np.array_equal(got, want), step
        torch.cuda.synchronize()
