"""The resident Session engine (compat/resident.py, csrc/bind_mlp.cpp
ResidentMLPPlan, csrc/kernels/mlp_persist_f32.hip RES): example.py's training
graph fed MNIST-loader batches keeps ONE persistent kernel launched across
Session.run calls.  Checked against an fp64 evaluation of the graph after
every step (loss, accuracy, global_step, parameters: relative 1e-5), across
idle exits / relaunches, interleaved variable writes (quiesce), a fallback
for non-one-hot labels, and global_step dtypes."""
import os
import sys
import time

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from test_lowering_cpu import _graph  # noqa: E402
from test_lowering_gpu import _ref_step, _rel  # noqa: E402

pytestmark = pytest.mark.gpu


def _batches(n, B, seed):
    from distributed_tensorflow_example_amd.data.mnist import PixelBatch

    rng = np.random.default_rng(seed)
    return [(PixelBatch.of(rng.integers(0, 256, (B, 784), dtype=np.uint8)),
             np.eye(10, dtype=np.float32)[rng.integers(0, 10, B)]) for _ in range(n)]


def _check_steps(tf, sess, g, params, batches, lr, act="sigmoid", stable=False, step0=0):
    for s, (bx, by) in enumerate(batches):
        params, ref_ce, ref_acc = _ref_step(params, np.asarray(bx), by, lr, act, stable)
        _, ce, acc, step = sess.run([g["train"], g["ce"], g["acc"], g["gs"]], feed_dict={g["x"]: bx, g["y_"]: by})
        assert abs(ce - ref_ce) <= 1e-5 * abs(ref_ce), (s, ce, ref_ce)
        assert abs(acc - ref_acc) < 1e-6, (s, acc, ref_acc)
        assert step == step0 + s + 1
        for got, want in zip(g["W"], params):
            assert _rel(got.numpy(), want) < 1e-5, s
    return params


@pytest.mark.parametrize("stable,act,B", [(False, "sigmoid", 100), (True, "relu", 64), (False, "sigmoid", 112)])
def test_resident_steps_match_fp64(monkeypatch, stable, act, B):
    monkeypatch.setenv("DTF_RESIDENT_IDLE_S", "2.0")
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L

    g = _graph(tf, stable, act)
    batches = _batches(6, B, 11)
    if act == "relu":
        batches = [(type(bx).of((np.asarray(bx.u8) // 20).astype(np.uint8)), by) for bx, by in batches]
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        params = [v.numpy().astype(np.float64) for v in g["W"]]
        _check_steps(tf, sess, g, params, batches, 0.5, act, stable)
        plan = L.plan_for(g["train"])
        assert plan.resident_steps == 6 and plan._rplan.plan.launches() == 1
    tf.reset_default_graph()


def test_resident_idle_exit_and_relaunch(monkeypatch):
    monkeypatch.setenv("DTF_RESIDENT_IDLE_S", "0.05")
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L

    g = _graph(tf)
    batches = _batches(6, 100, 5)
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        params = [v.numpy().astype(np.float64) for v in g["W"]]
        params = _check_steps(tf, sess, g, params, batches[:3], 0.5)
        time.sleep(0.4)                      # the launch exits by itself
        rp = L.plan_for(g["train"])._rplan.plan
        _check_steps(tf, sess, g, params, batches[3:], 0.5, step0=3)
        assert rp.launches() >= 2 and rp.runs() == 6
    tf.reset_default_graph()


def test_resident_quiesce_on_variable_writes(monkeypatch):
    """Variable.load and an op-by-op run between resident runs: the engine is
    stopped first, the write lands, the next run relaunches from it."""
    monkeypatch.setenv("DTF_RESIDENT_IDLE_S", "2.0")
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L
    from distributed_tensorflow_example_amd.compat import resident

    g = _graph(tf)
    batches = _batches(4, 100, 8)
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        params = [v.numpy().astype(np.float64) for v in g["W"]]
        params = _check_steps(tf, sess, g, params, batches[:2], 0.5)
        assert resident.any_live()
        new_b2 = np.linspace(-1, 1, 10).astype(np.float32)
        g["W"][3].load(new_b2, sess)              # quiesces, then writes
        assert not resident.any_live()
        params[3] = new_b2.astype(np.float64)
        params = _check_steps(tf, sess, g, params, batches[2:3], 0.5, step0=2)
        sess.run(g["gs"].assign(10.0))            # an op-by-op run: quiesced before it writes
        _check_steps(tf, sess, g, params, batches[3:], 0.5, step0=10)
        assert L.plan_for(g["train"])._rplan.plan.launches() == 3
    tf.reset_default_graph()


def test_non_one_hot_labels_fall_back(monkeypatch):
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L

    g = _graph(tf)
    (bx, by), = _batches(1, 100, 3)
    soft = (0.9 * by + 0.01).astype(np.float32)      # label smoothing: not one-hot
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        params = [v.numpy().astype(np.float64) for v in g["W"]]
        params, ref_ce, _ = _ref_step(params, np.asarray(bx), soft, 0.5, "sigmoid", False)
        _, ce = sess.run([g["train"], g["ce"]], feed_dict={g["x"]: bx, g["y_"]: soft})
        assert abs(ce - ref_ce) <= 1e-5 * abs(ref_ce)
        plan = L.plan_for(g["train"])
        assert plan.resident_steps == 0 and plan._cplan.steps() == 1
        for got, want in zip(g["W"], params):
            assert _rel(got.numpy(), want) < 1e-5
    tf.reset_default_graph()


@pytest.mark.parametrize("dtype", ["float32", "int64", "int32"])
def test_global_step_dtypes(dtype):
    import distributed_tensorflow_example_amd.compat as tf

    tf.reset_default_graph()
    dt = {"float32": tf.float32, "int64": tf.int64, "int32": tf.int32}[dtype]
    gs = tf.Variable(0, dtype=dt, trainable=False, name="global_step")
    x = tf.placeholder(tf.float32, [None, 784])
    y_ = tf.placeholder(tf.float32, [None, 10])
    W1 = tf.Variable(tf.random_normal([784, 100], seed=1))
    W2 = tf.Variable(tf.random_normal([100, 10], seed=2))
    b1, b2 = tf.Variable(tf.zeros([100])), tf.Variable(tf.zeros([10]))
    z3 = tf.add(tf.matmul(tf.nn.sigmoid(tf.add(tf.matmul(x, W1), b1)), W2), b2)
    ce = tf.reduce_mean(-tf.reduce_sum(y_ * tf.log(tf.nn.softmax(z3)), reduction_indices=[1]))
    train = tf.train.GradientDescentOptimizer(0.01).minimize(ce, global_step=gs)
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        for bx, by in _batches(3, 50, 1):
            _, step = sess.run([train, gs], feed_dict={x: bx, y_: by})
        assert int(step) == 3 and int(gs.numpy()) == 3
    tf.reset_default_graph()


def test_resident_alternating_batch_sizes(monkeypatch):
    """Alternating two batch sizes rebuilds the resident plan each time: the
    direct runner of the first size must not relaunch its stopped engine next to
    the live one (two persistent kernels on the same variables would lose
    updates).  Every step matches the fp64 evaluation."""
    monkeypatch.setenv("DTF_RESIDENT_IDLE_S", "2.0")
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import resident

    g = _graph(tf)
    b100, b64 = _batches(4, 100, 21), _batches(4, 64, 22)
    order = [b100[0], b100[1], b64[0], b100[2], b64[1], b64[2], b100[3], b64[3]]
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        params = [v.numpy().astype(np.float64) for v in g["W"]]
        for s, b in enumerate(order):
            params = _check_steps(tf, sess, g, params, [b], 0.5, step0=s)
            assert len(resident._LIVE) <= 1
    tf.reset_default_graph()
