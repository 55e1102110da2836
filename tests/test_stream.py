"""Streaming ImageNet ingest (data/stream.py): bounded host memory, per-rank sharding,
epochs, undecodable records skipped, ring-slot recycling after the feeder's copy, the
streamed mean, and ImageNetApp end to end on a tiny tar shard (CPU engine).
Reference behaviour: ImageNetApp.scala:60-76 (compressed minibatches, mean from them)."""
import io
import os
import tarfile

import numpy as np
import torch

from sparknet_amd.data.loaders import ImageNetLoader
from sparknet_amd.data.stream import StreamingJpegSource, streamed_mean


def _jpeg(value):
    from PIL import Image
    buf = io.BytesIO()
    Image.new("RGB", (20, 12), (value, 255 - value, value // 2)).save(buf, format="JPEG", quality=95)
    return buf.getvalue()


def _shards(root, n_files=2, per_file=10, bad=1):
    os.makedirs(root, exist_ok=True)
    labels = []
    k = 0
    for f in range(n_files):
        with tarfile.open(os.path.join(root, f"shard{f}.tar"), "w") as tf:
            for i in range(per_file):
                name = f"img{k:04d}.JPEG"
                data = b"not a jpeg" if (bad and k == 3) else _jpeg(10 * k % 250)
                ti = tarfile.TarInfo(name)
                ti.size = len(data)
                tf.addfile(ti, io.BytesIO(data))
                labels.append(f"{name} {k % 5}")
                k += 1
    lab = os.path.join(os.path.dirname(root), "labels.txt")
    with open(lab, "w") as f:
        f.write("\n".join(labels))
    return lab


def test_stream_epochs_sharding_and_bounded_ring(tmp_path):
    root = str(tmp_path / "train")
    lab = _shards(root)
    ld = ImageNetLoader(root, lab, size=(8, 8))
    src = StreamingJpegSource(ld, 4, (0, 1), slots=3, workers=3, epochs=2, pin=False)
    seen = []
    for x, y in src:
        assert x.shape == (4, 3, 8, 8) and x.dtype == torch.uint8 and y.dtype == torch.int32
        seen.append(y.clone())
    # 20 records, 1 undecodable -> 19 per epoch -> 4 full batches of 4 (the last 3 dropped)
    assert len(seen) == 9 and src.images_skipped == 2
    assert src.host_bytes() == 3 * (4 * 3 * 8 * 8 + 4 * 4)
    labels = torch.cat(seen).tolist()
    assert set(labels) <= set(range(5))
    src.close()
    # two ranks with >= world shard files: each rank reads only its own file
    got = []
    for r in range(2):
        s = StreamingJpegSource(ld, 3, (r, 2), slots=2, workers=2, epochs=1, pin=False)
        got.append(sum(int(y.numel()) for _, y in s))
        s.close()
    assert got == [9, 9]  # shard0: 10 records - 1 bad = 9; shard1: 10 -> 3 batches of 3


def test_stream_shuffle_buffer_is_a_permutation(tmp_path):
    root = str(tmp_path / "train")
    lab = _shards(root, n_files=1, per_file=16, bad=0)
    ld = ImageNetLoader(root, lab, size=(4, 4))
    plain = [y.clone() for _, y in StreamingJpegSource(ld, 4, slots=2, workers=2, epochs=1, pin=False)]
    shuf = [y.clone() for _, y in StreamingJpegSource(ld, 4, slots=2, workers=2, epochs=1, shuffle_buffer=8,
                                                     seed=3, pin=False)]
    a, b = torch.cat(plain).tolist(), torch.cat(shuf).tolist()
    assert sorted(a) == sorted(b) and a != b


def test_ring_slot_recycled_only_after_submit(tmp_path):
    root = str(tmp_path / "train")
    lab = _shards(root, n_files=1, per_file=12, bad=0)
    ld = ImageNetLoader(root, lab, size=(4, 4))
    src = StreamingJpegSource(ld, 2, slots=2, workers=1, epochs=None, pin=False)
    x0, _ = src.next_batch()
    x1, _ = src.next_batch()
    snap = x0.clone()
    import time
    time.sleep(0.3)  # the batcher has no free slot: x0 must stay intact until submitted
    assert torch.equal(snap, x0)
    src.submitted(x0, None)
    x2, _ = src.next_batch()
    assert x2.data_ptr() == x0.data_ptr()  # the recycled slot
    src.close()


def test_streamed_mean_matches_full_decode(tmp_path):
    root = str(tmp_path / "train")
    lab = _shards(root, bad=0)
    ld = ImageNetLoader(root, lab, size=(6, 6))
    m = streamed_mean(ld, 5, workers=2)
    imgs = np.stack([img for img, _ in ld])
    np.testing.assert_allclose(m, imgs.astype(np.float64).mean(0), rtol=1e-5)


def test_imagenet_app_streaming_cpu(tmp_path):
    from sparknet_amd.apps import imagenet_app
    root = str(tmp_path / "train")
    lab = _shards(root, n_files=1, per_file=6, bad=0)
    solver = imagenet_app.main(["--cpu", "--data", root, "--labels", lab, "--batch", "2", "--test-batch", "2",
                                "--tau", "1", "--rounds", "1", "--test-every", "0", "--model", "caffenet",
                                "--log-dir", str(tmp_path / "logs"), "--decode-workers", "2", "--ring-slots", "2",
                                "--shuffle-buffer", "0"])
    assert solver is not None and solver.iter == 1
