"""Row-sharded tables saved as TF partitioned variables and restored across
world sizes and partition counts (gloo ranks on CPU).

Layout checked against TF's Saver for a PartitionedVariable
(SaveSliceInfo + SaveV2 -> BundleWriter::AddSlice): full-name entry with one
TensorSliceProto per contiguous fixed_size_partitioner partition, data under
EncodeTensorNameSlice keys (byte-level golden tests: test_native_runtime.py)."""
import os
import socket
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS, DIM = 1003, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q, mode, prefix, nparts):
    try:
        sys.path.insert(0, REPO)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(ws), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        from distributed_tensorflow_example_amd import ckpt
        from distributed_tensorflow_example_amd.parallel import world as Wm
        from distributed_tensorflow_example_amd.parallel.sharded_embedding import ShardedEmbedding

        w = Wm.init(backend="gloo")
        t = ShardedEmbedding(ROWS, DIM, w, init_std=1.0, seed=11, name="emb/W")
        if mode == "save":
            with torch.no_grad():
                t.local.add_(0.25)                          # values independent of the world size
            path = ckpt.save_sharded(prefix, {"emb/W": t}, {"step": torch.tensor(5)}, w, num_partitions=nparts)
            q.put((rank, t.full_table().numpy(), path))
        else:
            with torch.no_grad():
                t.local.zero_()
            ckpt.restore_sharded(prefix, {"emb/W": t})
            q.put((rank, t.full_table().numpy(), t.local.numpy().copy()))
        w.shutdown()
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc(), None))


def _run(ws, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, ws, port, q) + args) for r in range(ws)]
    [p.start() for p in ps]
    out = sorted([q.get(timeout=240) for _ in range(ws)], key=lambda r: r[0])
    [p.join(60) for p in ps]
    for r in out:
        assert not isinstance(r[1], str), r[1]
    return out


def test_partitioned_save_three_ranks_restore_two_and_one(tmp_path):
    sys.path.insert(0, REPO)
    from distributed_tensorflow_example_amd import ckpt
    from distributed_tensorflow_example_amd.compat import saver

    prefix = str(tmp_path / "ck" / "m")
    saved = _run(3, "save", prefix, 5)              # 5 partitions over 3 ranks (rank k % 3 writes part k)
    full = saved[0][1]
    path = saved[0][2]
    idx = saver.read_bundle_index(path)
    ext = saver.partition_extents(ROWS, 5)
    assert ext == [(0, 201), (201, 201), (402, 201), (603, 200), (803, 200)]
    assert sorted(idx["emb/W"]["slices"]) == [[(a, n), (0, DIM)] for a, n in ext]
    assert idx["emb/W"]["shape"] == [ROWS, DIM] and idx["emb/W"]["size"] == 0
    assert all(os.path.exists(f"{path}.data-0000{r}-of-00003") for r in range(3))
    assert np.array_equal(saver.read_tensor(path, "emb/W").numpy(), full)
    for (a, n) in ext:
        assert np.array_equal(saver.read_slice(path, "emb/W", [(a, n), (0, DIM)]).numpy(), full[a:a + n])
    # restore on 2 ranks and on 1 rank: each keeps the rows it owns
    two = _run(2, "restore", path, None)
    assert np.array_equal(two[0][1], full) and np.array_equal(two[1][2], full[1::2])
    one = _run(1, "restore", path, None)
    assert np.array_equal(one[0][1], full)
    # a plain (unpartitioned) full entry restores into a sharded table too
    saver.write_bundle(str(tmp_path / "plain"), {"emb/W": torch.from_numpy(full)})
    two_plain = _run(2, "restore", str(tmp_path / "plain"), None)
    assert np.array_equal(two_plain[0][1], full)


def test_partition_extents_matches_fixed_size_partitioner():
    sys.path.insert(0, REPO)
    from distributed_tensorflow_example_amd.compat.saver import partition_extents

    for rows in (1, 7, 10, 1000, 4_700_000):
        for P in (1, 2, 3, 8, 16):
            ext = partition_extents(rows, P)
            sizes = [n for _, n in ext]
            assert sum(sizes) == rows and ext[0][0] == 0
            assert all(ext[i][0] + ext[i][1] == ext[i + 1][0] for i in range(len(ext) - 1))
            assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)
            assert len(ext) == min(P, rows)
