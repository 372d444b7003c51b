"""replica_device_setter path for big tables: a ps-placed tf.Variable becomes
a row-sharded PartitionedVariable; lr2.py's graph trains identically on 1
and 2 gloo workers; checkpoints hold TF's PartitionedVariable layout
(full-name entry + contiguous slices) and re-shard on restore."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F = 4000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


_OPTS = {"sgd": lambda tf: tf.train.GradientDescentOptimizer(0.5),
         "adagrad": lambda tf: tf.train.AdagradOptimizer(0.5),
         "adam": lambda tf: tf.train.AdamOptimizer(0.05),
         "momentum": lambda tf: tf.train.MomentumOptimizer(0.2, 0.9, use_nesterov=True),
         "rmsprop": lambda tf: tf.train.RMSPropOptimizer(0.05, momentum=0.5)}


def _graph(tf, opt="sgd"):
    with tf.device(tf.train.replica_device_setter(ps_tasks=1)):
        gs = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0), trainable=False)
        with tf.name_scope("input"):
            shp, idx = tf.placeholder(tf.int64), tf.placeholder(tf.int64)
            fid, fv = tf.placeholder(tf.int64), tf.placeholder(tf.float32)
            y = tf.placeholder(tf.float32, [None, 1])
            sp_f = tf.SparseTensor(shape=shp, indices=idx, values=fid)
            sp_v = tf.SparseTensor(shape=shp, indices=idx, values=fv)
        with tf.name_scope("weights"):
            W = tf.Variable(tf.random_normal([F, 1]))
        with tf.name_scope("bias"):
            b = tf.Variable(tf.zeros([1]))
        with tf.name_scope("loss"):
            py_x = tf.add(tf.nn.embedding_lookup_sparse(W, sp_f, sp_v, combiner="sum"), b)
            ce = tf.reduce_mean(tf.nn.sigmoid_cross_entropy_with_logits(py_x, y))
        train = _OPTS[opt](tf).minimize(ce, global_step=gs)
    return dict(gs=gs, shp=shp, idx=idx, fid=fid, fv=fv, y=y, W=W, b=b, train=train)


def _feed(g, batch):
    labels, fids, fvals, sp_indices, n = batch.as_tf_feed()
    return {g["y"]: labels, g["shp"]: np.array([F, n]), g["idx"]: sp_indices, g["fid"]: fids, g["fv"]: fvals}


def _worker(rank, ws, port, q, files, ckdir, mode="sync", opt="sgd"):
    try:
        sys.path.insert(0, REPO)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(ws), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port), DTF_SHARD_MIN_ROWS="1000", DTF_UPDATE_MODE=mode)
        import distributed_tensorflow_example_amd.compat as tf
        from distributed_tensorflow_example_amd.data import libsvm
        from distributed_tensorflow_example_amd.parallel import world as Wm

        w = Wm.init(backend="gloo")
        data = libsvm.load_files(files)
        tf.set_random_seed(7)
        g = _graph(tf, opt)
        assert type(g["W"]).__name__ == "PartitionedVariable"
        sv = tf.train.Supervisor(is_chief=(rank == 0), global_step=g["gs"], init_op=tf.global_variables_initializer())
        with sv.prepare_or_wait_for_session() as sess:
            for s in range(6):
                rows = np.arange(s * 200, (s + 1) * 200)[rank * 200 // ws:(rank + 1) * 200 // ws]
                sess.run(g["train"], feed_dict=_feed(g, data.take(rows)))
            full = g["W"].numpy().copy()
            bias = sess.run(g["b"]).copy()
            path = tf.train.Saver().save(sess, os.path.join(ckdir, f"ws{ws}_{opt}", "m"), global_step=g["gs"])
            step = float(sess.run(g["gs"]))
        q.put((rank, full, bias, path, step))
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc(), None, None, None))


def _run(ws, files, ckdir, mode="sync", opt="sgd"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, ws, port, q, files, ckdir, mode, opt)) for r in range(ws)]
    [p.start() for p in ps]
    out = sorted([q.get(timeout=240) for _ in range(ws)], key=lambda r: r[0])
    [p.join(60) for p in ps]
    for r in out:
        assert not isinstance(r[1], str), r[1]
    return out


def test_partitioned_variable_sync_workers(tmp_path):
    sys.path.insert(0, REPO)
    os.environ["DTF_SHARD_MIN_ROWS"] = "1000"
    from distributed_tensorflow_example_amd.data import libsvm

    files = libsvm.write_synthetic(str(tmp_path / "p"), 1, 1200, F, 10, seed=4)
    one = _run(1, files, str(tmp_path))
    two = _run(2, files, str(tmp_path))
    assert np.array_equal(two[0][1], two[1][1]) and np.array_equal(two[0][2], two[1][2])
    assert np.allclose(one[0][1], two[0][1], atol=1e-6)
    assert np.allclose(one[0][2], two[0][2], atol=1e-6)
    assert one[0][4] == two[0][4] == 6.0
    # 2-shard checkpoint restored into a 1-worker graph (re-sharding)
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.parallel import world as Wm

    Wm.reset()
    idx = tf.train.list_variables(os.path.dirname(two[0][3]))
    names = dict(idx)
    assert names["weights/Variable"] == [F, 1] and not any("part_" in k for k in names)
    from distributed_tensorflow_example_amd.compat import saver as S

    e = S.read_bundle_index(two[0][3])["weights/Variable"]
    assert e["slices"] == [[(0, F // 2), (0, 1)], [(F // 2, F // 2), (0, 1)]]   # one partition per worker
    assert np.array_equal(S.read_tensor(two[0][3], "weights/Variable").numpy(), two[0][1])
    tf.reset_default_graph()
    g = _graph(tf)
    with tf.Session() as sess:
        tf.train.Saver().restore(sess, two[0][3])
        assert np.allclose(g["W"].numpy(), two[0][1])
        assert float(sess.run(g["gs"])) == 6.0
    tf.reset_default_graph()


def test_restore_reads_the_old_modulo_part_layout(tmp_path):
    """Checkpoints of this repo's earlier layout (`W/part_k` = rows r % P == k)
    still restore: the table is rebuilt the modulo way."""
    import torch

    sys.path.insert(0, REPO)
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat.saver import write_bundle

    tf.reset_default_graph()
    g = _graph(tf)
    full = torch.arange(F, dtype=torch.float32).reshape(F, 1) * 0.5
    prefix = str(tmp_path / "old.ckpt")
    P = 3
    write_bundle(prefix, {**{f"weights/Variable/part_{k}": full[k::P].clone() for k in range(P)},
                          "bias/Variable": torch.tensor([2.5]), "global_step": torch.tensor(7.0)})
    saver = tf.train.Saver()
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        saver.restore(sess, prefix)
        w = sess.run(g["W"])
        assert np.array_equal(np.asarray(w).reshape(-1), full.numpy().reshape(-1))
        assert float(np.asarray(sess.run(g["b"])).reshape(-1)[0]) == 2.5
    # an incomplete old set is a clear error, not "variables not found"
    write_bundle(prefix, {"weights/Variable/part_0": full[0::3].clone(), "weights/Variable/part_2": full[2::3].clone(),
                          "bias/Variable": torch.tensor([2.5]), "global_step": torch.tensor(7.0)})
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        try:
            saver.restore(sess, prefix)
            raise AssertionError("restore of an incomplete part set must fail")
        except KeyError as e:
            assert "incomplete old-layout" in str(e)
    tf.reset_default_graph()


def test_partitioned_variable_async_workers(tmp_path):
    """lr2.py's graph with the reference's asynchronous rule (plain
    GradientDescentOptimizer under replica_device_setter, no SyncReplicas):
    the ps-placed W is a PartitionedVariable whose rows every worker reads from
    and scatter-updates into the owners' shared shards (HogwildTable) without
    waiting; global_step counts both workers' updates (2 x 6 = 12)."""
    sys.path.insert(0, REPO)
    os.environ["DTF_SHARD_MIN_ROWS"] = "1000"
    from distributed_tensorflow_example_amd.data import libsvm

    files = libsvm.write_synthetic(str(tmp_path / "p"), 1, 1200, F, 10, seed=4)
    one = _run(1, files, str(tmp_path))
    two = _run(2, files, str(tmp_path), "async")
    assert max(r[4] for r in two) == 12.0, [r[4] for r in two]     # the last update saw both workers' steps
    for r in two:
        assert np.isfinite(r[1]).all() and np.isfinite(r[2]).all()
    # ONE shared table: both workers read the same rows at the end (after the
    # collective save), and it trained (differs from a sync run of 6 steps)
    assert np.array_equal(two[0][1], two[1][1])
    assert not np.allclose(two[0][1], one[0][1])


import pytest  # noqa: E402


@pytest.mark.parametrize("opt,slots", [("adagrad", ["Adagrad"]), ("adam", ["Adam", "Adam_1"]),
                                       ("momentum", ["Momentum"]), ("rmsprop", ["RMSProp", "Momentum"])])
def test_partitioned_variable_sparse_optimizers(tmp_path, opt, slots):
    """Partitioned (ps-placed) variables under TF's other optimizers: the owner
    applies TF's sparse rule (duplicates summed, then Adagrad / Momentum /
    RMSProp per touched row; Adam's dense-decay _apply_sparse over the shard);
    1 and 2 workers agree, and the sharded slots are checkpointed in the TF
    slice layout (`weights/Variable/<slot>`) and re-shard on restore."""
    sys.path.insert(0, REPO)
    os.environ["DTF_SHARD_MIN_ROWS"] = "1000"
    from distributed_tensorflow_example_amd.data import libsvm

    files = libsvm.write_synthetic(str(tmp_path / "p"), 1, 1200, F, 10, seed=4)
    one = _run(1, files, str(tmp_path), opt=opt)
    two = _run(2, files, str(tmp_path), opt=opt)
    assert np.array_equal(two[0][1], two[1][1])
    assert np.allclose(one[0][1], two[0][1], atol=1e-5), np.abs(one[0][1] - two[0][1]).max()
    assert np.allclose(one[0][2], two[0][2], atol=1e-5)
    sgd = _run(1, files, str(tmp_path), opt="sgd")
    assert not np.allclose(one[0][1], sgd[0][1])           # a different rule really ran
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import saver as S
    from distributed_tensorflow_example_amd.parallel import world as Wm

    Wm.reset()
    idx = S.read_bundle_index(two[0][3])
    for sl in slots:
        e = idx[f"weights/Variable/{sl}"]
        assert e["slices"] == [[(0, F // 2), (0, 1)], [(F // 2, F // 2), (0, 1)]]
    one_slots = {sl: S.read_tensor(one[0][3], f"weights/Variable/{sl}").numpy() for sl in slots}
    for sl in slots:
        assert np.allclose(S.read_tensor(two[0][3], f"weights/Variable/{sl}").numpy(), one_slots[sl], atol=1e-5)
    # restore into a 1-worker graph: table and slots re-shard
    tf.reset_default_graph()
    g = _graph(tf, opt)
    with tf.Session() as sess:
        tf.train.Saver().restore(sess, two[0][3])
        assert np.allclose(g["W"].numpy(), two[0][1])
        for sl in slots:
            assert np.allclose(g["W"].table.slots[sl].cpu().numpy(), one_slots[sl], atol=1e-5)
    tf.reset_default_graph()
