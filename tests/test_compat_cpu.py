"""TF-1.x compat layer on CPU: graph/session semantics, TF variable naming and
placement, optimizers (vs closed-form TF update rules), Supervisor /
MonitoredTrainingSession + hooks, queues / input pipelines, streaming AUC,
sparse embedding lookup, flags, gfile (fake HDFS)."""
import os
import threading

import numpy as np
import pytest
import torch

import distributed_tensorflow_example_amd.compat as tf


@pytest.fixture(autouse=True)
def fresh_graph():
    tf.reset_default_graph()
    yield
    tf.reset_default_graph()


def test_names_scopes_and_placement():
    with tf.device(tf.train.replica_device_setter(ps_tasks=2, worker_device="/job:worker/task:1")):
        gs = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0), trainable=False)
        with tf.name_scope("weights"):
            w1 = tf.Variable(tf.random_normal([4, 3]))
            w2 = tf.Variable(tf.random_normal([3, 2]))
        x = tf.placeholder(tf.float32, [None, 4], name="x-input")
    assert [v.name for v in tf.global_variables()] == ["global_step:0", "weights/Variable:0", "weights/Variable_1:0"]
    assert [v.name for v in tf.trainable_variables()] == ["weights/Variable:0", "weights/Variable_1:0"]
    assert gs.placement == "/job:ps/task:0" and w1.placement == "/job:ps/task:1" and w2.placement == "/job:ps/task:0"
    assert x.name == "x-input:0"
    assert gs.dtype == torch.float32      # TF: get_variable default dtype


def test_session_feed_fetch_memoised():
    calls = []
    x = tf.placeholder(tf.float32, [None, 2])
    y = tf.Tensor(lambda a: (calls.append(1), a * 2)[1], [x], "dbl")
    z = y + 1
    with tf.Session() as sess:
        a, b, (c,) = sess.run([y, z, (y,)], feed_dict={x: np.ones((3, 2))})
        assert np.allclose(a, 2) and np.allclose(b, 3) and np.allclose(c, 2)
        assert len(calls) == 1
        d = sess.run({"k": z}, {x: np.zeros((1, 2))})
        assert np.allclose(d["k"], 1)
        with pytest.raises(KeyError):
            sess.run(z)
        f = sess.make_callable(z, [x])
        assert np.allclose(f(np.ones((1, 2))), 3)


def _mlp_graph(lr=0.5, opt="sgd"):
    tf.set_random_seed(1)
    x = tf.placeholder(tf.float32, [None, 784])
    y_ = tf.placeholder(tf.float32, [None, 10])
    with tf.name_scope("weights"):
        W1 = tf.Variable(tf.random_normal([784, 100]))
        W2 = tf.Variable(tf.random_normal([100, 10]))
    with tf.name_scope("biases"):
        b1 = tf.Variable(tf.zeros([100]))
        b2 = tf.Variable(tf.zeros([10]))
    a2 = tf.nn.sigmoid(tf.add(tf.matmul(x, W1), b1))
    y = tf.nn.softmax(tf.add(tf.matmul(a2, W2), b2))
    ce = tf.reduce_mean(-tf.reduce_sum(y_ * tf.log(y), reduction_indices=[1]))
    gs = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0), trainable=False)
    o = {"sgd": lambda: tf.train.GradientDescentOptimizer(lr),
         "adam": lambda: tf.train.AdamOptimizer(lr),
         "mom": lambda: tf.train.MomentumOptimizer(lr, 0.9)}[opt]()
    train_op = o.minimize(ce, global_step=gs)
    acc = tf.reduce_mean(tf.cast(tf.equal(tf.argmax(y, 1), tf.argmax(y_, 1)), tf.float32))
    return dict(x=x, y_=y_, W1=W1, W2=W2, b1=b1, b2=b2, ce=ce, gs=gs, train_op=train_op, acc=acc)


def test_gradient_descent_matches_reference_math():
    from distributed_tensorflow_example_amd.models import mlp

    g = _mlp_graph(lr=0.1)
    rng = np.random.default_rng(0)
    bx = rng.random((100, 784), dtype=np.float32)
    by = np.eye(10, dtype=np.float32)[rng.integers(0, 10, 100)]
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        p0 = {k: torch.tensor(sess.run(g[k])) for k in ("W1", "b1", "W2", "b2")}
        _, c = sess.run([g["train_op"], g["ce"]], {g["x"]: bx, g["y_"]: by})
        p1 = {k: torch.tensor(sess.run(g[k])) for k in ("W1", "b1", "W2", "b2")}
        assert float(sess.run(g["gs"])) == 1.0
    flat = torch.cat([p0["W1"].reshape(-1), p0["W2"].reshape(-1), p0["b1"], p0["b2"]])
    loss, _, gflat = mlp.reference_loss_and_grad(flat, torch.tensor(bx), torch.tensor(by.argmax(1)), naive=True)
    assert abs(float(loss) - float(c)) < 1e-4
    gd = mlp.unflatten(gflat)
    names = {"W1": "weights/Variable", "W2": "weights/Variable_1", "b1": "biases/Variable", "b2": "biases/Variable_1"}
    for k in p0:
        assert torch.allclose(p1[k], p0[k] - 0.1 * gd[names[k]], atol=1e-5)


def test_adam_tf_semantics_and_slots(tmp_path):
    x = tf.placeholder(tf.float32, [None, 1])
    yv = tf.placeholder(tf.float32, [None, 1])
    with tf.variable_scope("test"):
        w = tf.get_variable("weights", [1, 1], initializer=tf.constant_initializer(0.5))
        b = tf.get_variable("bias", [1], initializer=tf.constant_initializer(0.0))
    pred = tf.matmul(x, w) + b
    loss = tf.reduce_sum(tf.pow(yv - pred, 2)) / 10
    train = tf.train.AdamOptimizer(0.01).minimize(loss)
    names = {v.name for v in tf.global_variables()}
    assert {"test/weights/Adam:0", "test/weights/Adam_1:0", "beta1_power:0", "beta2_power:0"} <= names
    xs = np.arange(10, dtype=np.float32).reshape(10, 1)
    ys = 2 * xs + 1
    # closed-form TF Adam
    wt, bt = np.array([[0.5]]), np.array([0.0])
    m = [np.zeros_like(wt), np.zeros_like(bt)]
    v = [np.zeros_like(wt), np.zeros_like(bt)]
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        for t in range(1, 6):
            sess.run(train, {x: xs, yv: ys})
            r = ys - (xs @ wt + bt)
            gw, gb = -2 * xs.T @ r / 10, -2 * r.sum(0) / 10
            lr_t = 0.01 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
            for i, (p, gg) in enumerate(((wt, gw), (bt, gb))):
                m[i] = 0.9 * m[i] + 0.1 * gg
                v[i] = 0.999 * v[i] + 0.001 * gg * gg
                p -= lr_t * m[i] / (np.sqrt(v[i]) + 1e-8)
        assert np.allclose(sess.run(w), wt, atol=1e-6) and np.allclose(sess.run(b), bt, atol=1e-6)
        path = tf.train.Saver().save(sess, str(tmp_path / "model.ckpt"))
    r = tf.train.NewCheckpointReader(path)
    assert r.has_tensor("test/weights/Adam_1") and abs(float(r.get_tensor("beta1_power")) - 0.9 ** 6) < 1e-6


def test_supervisor_trains_and_checkpoints(tmp_path):
    from distributed_tensorflow_example_amd.data import mnist

    ds = mnist.read_data_sets("", one_hot=True, train_size=2000, test_size=500)
    g = _mlp_graph(lr=0.05)
    tf.summary.scalar("cost", g["ce"])
    summary_op = tf.summary.merge_all()
    init = tf.global_variables_initializer()
    sv = tf.train.Supervisor(is_chief=True, logdir=str(tmp_path), global_step=g["gs"], init_op=init,
                             summary_op=None, save_model_secs=0)
    costs = []
    with sv.managed_session() as sess:
        for _ in range(60):
            bx, by = ds.train.next_batch(100)
            _, c, s, step = sess.run([g["train_op"], g["ce"], summary_op, g["gs"]], {g["x"]: bx, g["y_"]: by})
            sv.summary_computed(sess, s, int(step))
            costs.append(float(c))
    assert np.mean(costs[-10:]) < np.mean(costs[:10])
    ck = tf.train.latest_checkpoint(str(tmp_path))
    assert ck and ck.endswith("-60")
    assert any("tfevents" in f for f in os.listdir(tmp_path))
    # a fresh graph resumes from the checkpoint
    tf.reset_default_graph()
    g2 = _mlp_graph(lr=0.05)
    sv2 = tf.train.Supervisor(is_chief=True, logdir=str(tmp_path), global_step=g2["gs"], save_model_secs=0)
    with sv2.managed_session() as sess:
        assert float(sess.run(g2["gs"])) == 60.0
        w = sess.run(g2["W1"])
    assert np.allclose(w, tf.train.load_variable(ck, "weights/Variable"))


def test_monitored_training_session_hooks(tmp_path):
    from distributed_tensorflow_example_amd.data import mnist

    ds = mnist.read_data_sets("", one_hot=True, train_size=1000, test_size=100)
    g = _mlp_graph(lr=0.05, opt="mom")
    tf.summary.scalar("cost", g["ce"])
    seen = []

    class Rec(tf.train.SessionRunHook):
        def after_run(self, ctx, vals):
            seen.append(1)
    hooks = [tf.train.StopAtStepHook(last_step=25), tf.train.NanTensorHook(g["ce"]), Rec(),
             tf.train.LoggingTensorHook({"loss": g["ce"]}, every_n_iter=10)]
    n = 0
    with tf.train.MonitoredTrainingSession(is_chief=True, checkpoint_dir=str(tmp_path), hooks=hooks,
                                           save_checkpoint_steps=10, save_summaries_steps=5,
                                           log_step_count_steps=10) as mon:
        while not mon.should_stop():
            bx, by = ds.train.next_batch(50)
            mon.run(g["train_op"], {g["x"]: bx, g["y_"]: by})
            n += 1
    assert n == 25 and len(seen) == 25
    assert tf.train.latest_checkpoint(str(tmp_path)).endswith("-25")
    evs = [f for f in os.listdir(tmp_path) if "tfevents" in f]
    assert evs


def test_nan_hook_raises():
    v = tf.Variable(tf.constant([1.0]))
    bad = tf.log(v - 1.0) * 0.0 + tf.log(v - 2.0)
    with pytest.raises(tf.train.NanLossDuringTrainingError):
        with tf.train.MonitoredTrainingSession(hooks=[tf.train.NanTensorHook(bad)]) as mon:
            mon.run(bad)


def test_fifo_queue_batch_and_timeout():
    q = tf.FIFOQueue(capacity=50, dtypes=[tf.float32, tf.float32], shapes=[[4], [3]])
    xs = tf.placeholder(tf.float32, [None, 4])
    ys = tf.placeholder(tf.float32, [None, 3])
    enq = q.enqueue_many([xs, ys])
    bx, by = tf.train.batch(q.dequeue(), batch_size=15, capacity=40)
    data = np.arange(400, dtype=np.float32).reshape(100, 4)
    lab = np.tile(np.array([[1, 0, 0]], np.float32), (100, 1))
    with tf.Session() as sess:
        coord = tf.train.Coordinator()

        def feeder():
            for i in range(0, 100, 20):
                sess.run(enq, {xs: data[i:i + 20], ys: lab[i:i + 20]})
        t = threading.Thread(target=feeder, daemon=True)
        t.start()
        threads = tf.train.start_queue_runners(sess, coord)
        out = [sess.run([bx, by], options=tf.RunOptions(timeout_in_ms=4000)) for _ in range(6)]
        assert out[0][0].shape == (15, 4) and out[0][1].shape == (15, 3)
        got = np.concatenate([o[0] for o in out])
        assert np.array_equal(got, data[:90])
        with pytest.raises(tf.errors.DeadlineExceededError):
            sess.run(bx, options=tf.RunOptions(timeout_in_ms=300))
        coord.request_stop()
        sess.run(q.close(cancel_pending_enqueues=True))
        coord.join(threads, stop_grace_period_secs=5)


def test_slice_input_producer_and_dynamic_partition(tmp_path):
    files = []
    for i in range(6):
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(bytes([i]) * 3)
        files.append(str(p))
    labels = list(range(6))
    part = [0, 1, 0, 0, 1, 0]
    tr_f, te_f = tf.dynamic_partition(files, part, 2)
    tr_l, te_l = tf.dynamic_partition(labels, part, 2)
    fname, lab = tf.train.slice_input_producer([tr_f, tr_l], shuffle=False)
    content = tf.read_file(fname)
    bc, bl = tf.train.batch([content, lab], batch_size=2)
    with tf.Session() as sess:
        coord = tf.train.Coordinator()
        th = tf.train.start_queue_runners(sess, coord)
        c, l = sess.run([bc, bl])
        assert list(l) == [0, 2]
        assert [bytes(x) for x in c] == [b"\x00" * 3, b"\x02" * 3]
        coord.request_stop()
        coord.join(th, stop_grace_period_secs=5)


def test_streaming_auc_and_local_init():
    pred = tf.placeholder(tf.float32, [None])
    lab = tf.placeholder(tf.float32, [None])
    auc, upd = tf.contrib.metrics.streaming_auc(pred, lab)
    rng = np.random.default_rng(0)
    with tf.Session() as sess:
        sess.run(tf.local_variables_initializer())
        ps, ls = [], []
        for _ in range(5):
            l = (rng.random(2000) > 0.6).astype(np.float32)
            p = 1 / (1 + np.exp(-(rng.standard_normal(2000) + 1.2 * l)))
            sess.run(upd, {pred: p, lab: l})
            ps.append(p)
            ls.append(l)
        a = float(sess.run(auc))
    p, l = np.concatenate(ps), np.concatenate(ls)
    r = p.argsort().argsort() + 1
    P = l.sum()
    exact = (r[l > 0].sum() - P * (P + 1) / 2) / (P * (len(l) - P))
    assert abs(a - exact) < 5e-3


def _tf_streaming_auc_numpy(p, l, T=200):
    """TF contrib.metrics.streaming_auc from its definition (thresholds, confusion
    counts at p > t, compute_auc with epsilon 1e-6), in numpy fp32."""
    t = np.array([0.0 - 1e-7] + [(i + 1) * 1.0 / (T - 1) for i in range(T - 2)] + [1.0 + 1e-7], np.float32)
    above = p.astype(np.float32)[None, :] > t[:, None]
    pos = l.astype(bool)[None, :]
    tp = (above & pos).sum(1).astype(np.float32)
    fn = (~above & pos).sum(1).astype(np.float32)
    tn = (~above & ~pos).sum(1).astype(np.float32)
    fp = (above & ~pos).sum(1).astype(np.float32)
    e = np.float32(1e-6)
    rec = (tp + e) / (tp + fn + e)
    fpr = fp / (fp + tn + e)
    return float(np.sum((fpr[:-1] - fpr[1:]) * (rec[:-1] + rec[1:]) / np.float32(2.0))), (tp, fn, tn, fp)


def test_streaming_auc_tf_semantics():
    """TF variable names, exact TF thresholds / compute_auc, update_op = post-update
    value, value fetched with the update = pre-update value."""
    pred = tf.placeholder(tf.float32, [None])
    lab = tf.placeholder(tf.float32, [None])
    auc, upd = tf.contrib.metrics.streaming_auc(pred, lab)
    names = sorted(v.name for v in tf.local_variables() if v.name.startswith("auc"))
    assert names == ["auc/false_negatives:0", "auc/false_positives:0", "auc/true_negatives:0",
                     "auc/true_positives:0"]
    rng = np.random.default_rng(1)
    batches = []
    for _ in range(3):
        l = (rng.random(700) > 0.5).astype(np.float32)
        p = rng.random(700).astype(np.float32)
        p[:5] = [0.0, 1.0, 0.5, 1.0 / 199, 198.0 / 199]      # on / next to thresholds
        batches.append((p, l))
    with tf.Session() as sess:
        sess.run(tf.local_variables_initializer())
        seen_p, seen_l = [], []
        for p, l in batches:
            before = _tf_streaming_auc_numpy(np.concatenate(seen_p), np.concatenate(seen_l))[0] if seen_p else None
            v_pre, v_post = sess.run([auc, upd], {pred: p, lab: l})
            seen_p.append(p)
            seen_l.append(l)
            ref, (tp, fn, tn, fp) = _tf_streaming_auc_numpy(np.concatenate(seen_p), np.concatenate(seen_l))
            assert abs(float(v_post) - ref) < 1e-6, (float(v_post), ref)
            if before is not None:
                assert abs(float(v_pre) - before) < 1e-6
            # fetch order does not change what the value tensor reports in that run
        v_post2, v_pre2 = sess.run([upd, auc], {pred: batches[0][0], lab: batches[0][1]})
        assert abs(float(v_pre2) - ref) < 1e-6
        got = {v.name: v.value.numpy() for v in tf.local_variables() if v.name.startswith("auc")}
    seen_p.append(batches[0][0])
    seen_l.append(batches[0][1])
    _, (tp, fn, tn, fp) = _tf_streaming_auc_numpy(np.concatenate(seen_p), np.concatenate(seen_l))
    np.testing.assert_array_equal(got["auc/true_positives:0"], tp)
    np.testing.assert_array_equal(got["auc/false_negatives:0"], fn)
    np.testing.assert_array_equal(got["auc/true_negatives:0"], tn)
    np.testing.assert_array_equal(got["auc/false_positives:0"], fp)


def test_embedding_lookup_sparse_lr_graph():
    """lr2.py model: W[F,1], sum combiner over (fid, fval), sigmoid xent, SGD."""
    F = 50
    y = tf.placeholder(tf.float32, [None, 1])
    sp_idx = tf.placeholder(tf.int64)
    sp_ids = tf.placeholder(tf.int64)
    sp_vals = tf.placeholder(tf.float32)
    sp_shape = tf.placeholder(tf.int64)
    W = tf.Variable(tf.random_normal([F, 1], seed=3))
    b = tf.Variable(tf.zeros([1]))
    ids_t = tf.SparseTensor(indices=sp_idx, values=sp_ids, shape=sp_shape)
    val_t = tf.SparseTensor(indices=sp_idx, values=sp_vals, shape=sp_shape)
    py_x = tf.nn.embedding_lookup_sparse(W, ids_t, val_t, combiner="sum") + b
    loss = tf.reduce_mean(tf.nn.sigmoid_cross_entropy_with_logits(py_x, y))
    train = tf.train.GradientDescentOptimizer(0.5).minimize(loss)
    rows = [[1, 5], [2], [7, 8, 9]]
    vals = [[1.0, 0.5], [2.0], [1.0, 1.0, -1.0]]
    idx = np.array([[r, f] for r, fs in enumerate(rows) for f in fs], np.int64)
    fid = np.array([f for fs in rows for f in fs], np.int64)
    fv = np.array([v for vs in vals for v in vs], np.float32)
    yl = np.array([[1], [0], [1]], np.float32)
    feed = {y: yl, sp_idx: idx, sp_ids: fid, sp_vals: fv, sp_shape: np.array([F, 3])}
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        W0 = sess.run(W).copy()
        out = sess.run(py_x, feed)
        exp = np.array([[W0[1, 0] + 0.5 * W0[5, 0]], [2 * W0[2, 0]], [W0[7, 0] + W0[8, 0] - W0[9, 0]]])
        assert np.allclose(out, exp, atol=1e-6)
        l0 = sess.run(loss, feed)
        for _ in range(20):
            sess.run(train, feed)
        assert sess.run(loss, feed) < l0
        assert np.allclose(sess.run(W)[[0, 3, 4, 6]], W0[[0, 3, 4, 6]])    # untouched rows


def test_flags_parsing():
    from distributed_tensorflow_example_amd.utils import flags

    fv = flags._FlagValues()
    flags.DEFINE_string("job_name", "", "ps or worker", flag_values=fv)
    flags.DEFINE_integer("task_index", 0, "", flag_values=fv)
    flags.DEFINE_float("learning_rate", 0.01, "", flag_values=fv)
    flags.DEFINE_boolean("sync", False, "", flag_values=fv)
    rest = fv(["prog", "--job_name=worker", "--task_index", "3", "--learning_rate=0.5", "--sync", "extra"])
    assert fv.job_name == "worker" and fv.task_index == 3 and fv.learning_rate == 0.5 and fv.sync is True
    assert rest == ["prog", "extra"]
    fv.work_dir = "/tmp/x"          # attribute assignment as config (lr2.py:300)
    assert fv.work_dir == "/tmp/x"


def test_gfile_fake_hdfs(tmp_path, monkeypatch):
    from distributed_tensorflow_example_amd.utils import gfile

    monkeypatch.setenv("DTF_FAKE_HDFS_ROOT", str(tmp_path))
    gfile._FS_CACHE.clear() if hasattr(gfile, "_FS_CACHE") else None
    gfile.MakeDirs("hdfs://nn:9000/data/train")
    with gfile.GFile("hdfs://nn:9000/data/train/part-0", "w") as f:
        f.write("1 3:1\n0 4:1\n")
    assert gfile.Exists("hdfs://nn:9000/data/train/part-0")
    assert (tmp_path / "data/train/part-0").exists()
    with gfile.GFile("hdfs://nn:9000/data/train/part-0") as f:
        assert [l for l in f] == ["1 3:1\n", "0 4:1\n"]
    assert gfile.Glob("hdfs://nn:9000/data/train/part-*") == ["hdfs://nn:9000/data/train/part-0"]
    assert tf.gfile.ListDirectory("hdfs://nn:9000/data/train") == ["part-0"]


def test_adagrad_rmsprop_tf_semantics():
    """Fused Adagrad / RMSProp follow TF's ApplyAdagrad / ApplyRMSProp (accumulator
    0.1, mean-square slot initialised to 1), slots named like TF's."""
    import distributed_tensorflow_example_amd.compat as tf

    for kind in ("adagrad", "rmsprop"):
        tf.reset_default_graph()
        w = tf.Variable(tf.constant([1.0, -2.0, 3.0]), name="w")
        x = tf.placeholder(tf.float32, [3])
        loss = tf.reduce_sum(w * w * x)
        opt = tf.train.AdagradOptimizer(0.1) if kind == "adagrad" else tf.train.RMSPropOptimizer(0.01, 0.9, 0.5)
        train = opt.minimize(loss)
        names = [v.name for v in tf.global_variables()]
        assert ("w/Adagrad:0" in names) if kind == "adagrad" else ({"w/RMSProp:0", "w/Momentum:0"} <= set(names))
        wv = np.array([1.0, -2.0, 3.0])
        acc, ms, mom = np.full(3, 0.1), np.ones(3), np.zeros(3)
        xs = np.array([0.5, 1.0, 2.0], np.float32)
        with tf.Session() as sess:
            sess.run(tf.global_variables_initializer())
            for _ in range(3):
                sess.run(train, feed_dict={x: xs})
                g = 2 * wv * xs
                if kind == "adagrad":
                    acc = acc + g * g
                    wv = wv - 0.1 * g / np.sqrt(acc)
                else:
                    ms = 0.9 * ms + 0.1 * g * g
                    mom = 0.5 * mom + 0.01 * g / np.sqrt(ms + 1e-10)
                    wv = wv - mom
            assert np.allclose(sess.run(w), wv, rtol=1e-5, atol=1e-6)
    tf.reset_default_graph()
