"""The lowered reference training graph on the GPU (compat/lowering.py +
csrc/kernels/graph_mlp.hip) against an fp64 evaluation of the same graph:
losses, accuracies, global_step and the parameters after every step agree
to fp32 rounding (relative 1e-5); other optimizers go through the kernels'
gradient mode; fetch sets that read interior nodes fall back to eager."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from test_lowering_cpu import _graph  # noqa: E402

pytestmark = pytest.mark.gpu


def _data(B, seed):
    rng = np.random.default_rng(seed)
    bx = (rng.integers(0, 256, (B, 784)) / 255.0).astype(np.float32)
    by = np.eye(10, dtype=np.float32)[rng.integers(0, 10, B)]
    return bx, by


def _ref_step(params, bx, by, lr, act, stable):
    """One SGD step of the graph in fp64 (autograd through the literal ops)."""
    W1, W2, b1, b2 = [torch.tensor(p, dtype=torch.float64, requires_grad=True) for p in params]
    x, y_ = torch.tensor(bx, dtype=torch.float64), torch.tensor(by, dtype=torch.float64)
    a2 = torch.sigmoid(x @ W1 + b1) if act == "sigmoid" else torch.relu(x @ W1 + b1)
    z3 = a2 @ W2 + b2
    y = torch.softmax(z3, 1)
    ce = (-(y_ * torch.log_softmax(z3, 1)).sum(1)).mean() if stable else (-(y_ * torch.log(y)).sum(1)).mean()
    acc = (y.argmax(1) == y_.argmax(1)).double().mean()
    ce.backward()
    new = [(p - lr * p.grad).detach().numpy() for p in (W1, W2, b1, b2)]
    return new, float(ce), float(acc)


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("stable,act,B", [(False, "sigmoid", 100), (False, "relu", 37), (True, "sigmoid", 128)])
def test_lowered_sgd_steps_match_fp64(stable, act, B):
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L

    g = _graph(tf, stable, act)
    lr = 0.5
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        params = [v.numpy().astype(np.float64) for v in g["W"]]
        for s in range(4):
            bx, by = _data(B, s)
            if act == "relu":
                bx *= 0.05            # keep relu logits finite in fp32 (TF fp32 gives NaN there too)
            params, ref_ce, ref_acc = _ref_step(params, bx, by, lr, act, stable)
            _, ce, acc, step = sess.run([g["train"], g["ce"], g["acc"], g["gs"]],
                                        feed_dict={g["x"]: bx, g["y_"]: by})
            assert abs(ce - ref_ce) <= 1e-5 * abs(ref_ce), (s, ce, ref_ce)
            assert abs(acc - ref_acc) < 1e-6
            assert step == s + 1
            for got, want in zip(g["W"], params):
                assert _rel(got.numpy(), want) < 1e-5
        plan = L.plan_for(g["train"])
        assert plan is not None and plan.steps == 4          # every run went through the kernels
        assert plan._cplan.steps() == 4                      # ... as one native call + graph replay each
    tf.reset_default_graph()


@pytest.mark.parametrize("opt", ["momentum", "adam"])
def test_gradient_mode_matches_eager(opt):
    """Optimizers other than one-worker SGD: the kernels write the gradients
    into the all-reduce bucket, the fused optimizer applies them.  Momentum is
    linear in the gradient, so params agree to fp32 rounding; Adam divides by
    sqrt(v) and amplifies rounding of near-zero gradients up to lr per step,
    so it is held to the losses and an lr-sized bound."""
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L

    out = {}
    for mode in ("1", "0"):
        os.environ["DTF_GRAPH_LOWERING"] = mode
        try:
            g = _graph(tf, opt=opt)
            with tf.Session() as sess:
                sess.run(tf.global_variables_initializer())
                ces = []
                for s in range(3):
                    bx, by = _data(64, 10 + s)
                    ces.append(sess.run([g["train"], g["ce"]], feed_dict={g["x"]: bx, g["y_"]: by})[1])
                out[mode] = ([v.numpy().copy() for v in g["W"]], ces, int(sess.run(g["gs"])))
                if mode == "1":
                    assert L.plan_for(g["train"]).steps == 3
        finally:
            os.environ.pop("DTF_GRAPH_LOWERING", None)
    (p1, c1, s1), (p0, c0, s0) = out["1"], out["0"]
    assert s1 == s0 == 3
    np.testing.assert_allclose(c1, c0, rtol=1e-5)
    for a, b in zip(p1, p0):
        if opt == "momentum":
            assert _rel(a, b) < 1e-5
        else:
            assert np.abs(a - b).max() <= 3 * 0.01 * 2
    tf.reset_default_graph()


def test_fetching_interior_node_falls_back():
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L

    g = _graph(tf)
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        params = [v.numpy().astype(np.float64) for v in g["W"]]
        bx, by = _data(50, 3)
        new, ref_ce, _ = _ref_step(params, bx, by, 0.5, "sigmoid", False)
        _, y, ce = sess.run([g["train"], g["y"], g["ce"]], feed_dict={g["x"]: bx, g["y_"]: by})
        assert abs(ce - ref_ce) <= 1e-5 * abs(ref_ce)
        for got, want in zip(g["W"], new):
            assert _rel(got.numpy(), want) < 1e-5
        plan = L.plan_for(g["train"])
        assert plan is not None and plan.steps == 0
    tf.reset_default_graph()


def test_lr2_graph_lowered_matches_op_by_op(monkeypatch):
    """lr2.py's graph (partitioned W, SparseTensor feeds, embedding_lookup_sparse
    + b, sigmoid xent, SGD): the lowered train run (native sparse-LR step
    replayed from hipGraphs per padded shape) trains like the op-by-op run."""
    monkeypatch.setenv("DTF_SHARD_MIN_ROWS", "1000")
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering

    F, B = 20000, 64
    rng = np.random.default_rng(5)
    feeds_np = []
    for _ in range(5):
        k = rng.integers(3, 12, size=B)
        rows = np.repeat(np.arange(B), k)
        ids = rng.integers(0, F, rows.size).astype(np.int64)
        feeds_np.append((np.stack([rows, ids], 1), ids, rng.random(rows.size).astype(np.float32),
                         (rng.random((B, 1)) < 0.4).astype(np.float32)))
    results = []
    for lower in ("1", "0"):
        monkeypatch.setenv("DTF_GRAPH_LOWERING", lower)
        tf.reset_default_graph()
        with tf.device(tf.train.replica_device_setter(ps_tasks=1)):
            gs = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0), trainable=False)
            shp, idx, fid, fv = (tf.placeholder(tf.int64), tf.placeholder(tf.int64), tf.placeholder(tf.int64),
                                 tf.placeholder(tf.float32))
            y = tf.placeholder(tf.float32, [None, 1])
            with tf.name_scope("weights"):
                W = tf.Variable(tf.random_normal([F, 1]))
            with tf.name_scope("bias"):
                b = tf.Variable(tf.zeros([1]))
            py_x = tf.add(tf.nn.embedding_lookup_sparse(W, tf.SparseTensor(shape=shp, indices=idx, values=fid),
                                                        tf.SparseTensor(shape=shp, indices=idx, values=fv),
                                                        combiner="sum"), b)
            ce = tf.reduce_mean(tf.nn.sigmoid_cross_entropy_with_logits(py_x, y))
            train = tf.train.GradientDescentOptimizer(0.5).minimize(ce, global_step=gs)
        assert W.table.local.is_cuda
        losses = []
        with tf.Session() as sess:
            sess.run(tf.global_variables_initializer())
            for s in range(12):
                i, f, v, lab = feeds_np[s % 5]
                _, l = sess.run([train, ce], feed_dict={shp: [F, B], idx: i, fid: f, fv: v, y: lab})
                losses.append(float(l))
            results.append((W.numpy().copy(), float(sess.run(b)[0]), float(sess.run(gs)), losses))
        plan = lowering.plan_for(train)
        assert (plan is not None and plan.steps == 12) == (lower == "1")
    (wl, bl, gl, ll), (we, be, ge, le) = results
    assert gl == ge == 12.0
    np.testing.assert_allclose(ll, le, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(wl, we, rtol=1e-5, atol=1e-5)
    assert abs(bl - be) < 1e-5


def test_uint8_feed_is_bit_identical(native):
    """GraphStepPlan.run_u8 (the MNIST loader's uint8 source of a PixelBatch,
    converted on the GPU with the loader's float32 division) vs run() with the
    float32 batch: identical metrics and parameters, bit for bit."""
    from distributed_tensorflow_example_amd.data.mnist import PixelBatch

    K, H, C, B = 784, 100, 10, 100
    g = torch.Generator(device="cpu").manual_seed(0)
    p0 = [torch.randn(K, H, generator=g) * 0.05, torch.zeros(H), torch.randn(H, C, generator=g) * 0.1, torch.zeros(C)]
    pa = [t.cuda().contiguous() for t in p0]
    pb = [t.cuda().contiguous() for t in p0]
    plan_f = native.GraphStepPlan(*pa, None, B, 0, True, False)
    plan_u = native.GraphStepPlan(*pb, None, B, 0, True, False)
    rng = np.random.default_rng(1)
    for _ in range(5):
        u8 = rng.integers(0, 256, (B, K), dtype=np.uint8)
        x = PixelBatch.of(u8)
        y = np.eye(C, dtype=np.float32)[rng.integers(0, C, B)]
        plan_f.run(np.asarray(x), y, 0.5, True)
        plan_u.run_u8(x.u8, y, 0.5, True)
        assert np.array_equal(plan_f.host_metrics().numpy(), plan_u.host_metrics().numpy())
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)


def test_session_uses_uint8_feed_for_loader_batches(monkeypatch):
    """examples/mnist_example.py's graph fed by the MNIST loader: the lowered
    plan takes the uint8 path and matches a float-fed session bit for bit
    (the launched plan's uint8 path: the resident engine is off here, it has
    tests of its own in test_resident_gpu.py)."""
    monkeypatch.setenv("DTF_RESIDENT_SESSION", "0")
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L
    from distributed_tensorflow_example_amd.data.mnist import PixelBatch

    rng = np.random.default_rng(3)
    batches = [(PixelBatch.of(rng.integers(0, 256, (100, 784), dtype=np.uint8)),
                np.eye(10, dtype=np.float32)[rng.integers(0, 10, 100)]) for _ in range(3)]
    finals = []
    for use_u8 in (True, False):
        g = _graph(tf)
        with tf.Session() as sess:
            sess.run(tf.global_variables_initializer())
            init = [v.numpy().copy() for v in g["W"]]
            if finals:
                for v, w in zip(g["W"], finals[0][0]):
                    v.load(w, sess)
            for bx, by in batches:
                sess.run([g["train"], g["ce"]], feed_dict={g["x"]: bx if use_u8 else np.array(bx), g["y_"]: by})
            plan = L.plan_for(g["train"])
            assert plan is not None and plan._cplan.steps() == 3
            finals.append((init, [v.numpy().copy() for v in g["W"]]))
        tf.reset_default_graph()
    for a, b in zip(finals[0][1], finals[1][1]):
        assert np.array_equal(a, b)


def test_loader_batches_with_captured_graph_plan(monkeypatch):
    """DTF_GRAPH_STEP_HIPGRAPH=1 builds the captured-graph plan, which takes
    float32 feeds only: loader PixelBatches must take its float path (not
    run_u8, which that plan refuses) and still train like the fp64 graph."""
    monkeypatch.setenv("DTF_GRAPH_STEP_HIPGRAPH", "1")
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L
    from distributed_tensorflow_example_amd.data.mnist import PixelBatch

    rng = np.random.default_rng(4)
    g = _graph(tf)
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        params = [v.numpy().astype(np.float64) for v in g["W"]]
        for s in range(3):
            bx = PixelBatch.of(rng.integers(0, 256, (100, 784), dtype=np.uint8))
            by = np.eye(10, dtype=np.float32)[rng.integers(0, 10, 100)]
            params, ref_ce, _ = _ref_step(params, np.asarray(bx), by, 0.5, "sigmoid", False)
            _, ce = sess.run([g["train"], g["ce"]], feed_dict={g["x"]: bx, g["y_"]: by})
            assert abs(ce - ref_ce) <= 1e-5 * abs(ref_ce)
        plan = L.plan_for(g["train"])
        assert plan is not None and plan._cplan.use_graph() and plan._cplan.steps() == 3
        for got, want in zip(g["W"], params):
            assert _rel(got.numpy(), want) < 1e-5
    tf.reset_default_graph()
