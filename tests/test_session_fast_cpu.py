"""Session.run's direct runner for a lowered plan (compat/session.py _fast,
compat/lowering.py SparseLRStepPlan.fast_runner): after one run of a fetch
list went through the one-GPU native sparse-LR call, the next runs of the same
fetch list hand the feed arrays straight to it.  The native plan is replaced
by a recorder and the table reports a GPU device, so the wiring is checked on
the CPU: calls, counters, the loss fetch, and the fall-back to the full path
for feeds the runner does not take."""
import numpy as np
import torch


class _Plan:
    def __init__(self, *a):
        self.calls = []

    def run(self, y, idx, ids, vals, lr):
        self.calls.append((y, ids, lr))
        return True

    def loss(self):
        return torch.tensor(0.25)


class _Native:
    SparseLRPlan = _Plan

    def __init__(self, real):
        self._real = real

    def __getattr__(self, k):
        return getattr(self._real, k)


class _Dev:
    type = "cuda"


def test_sparse_lr_fast_runner(monkeypatch):
    monkeypatch.setenv("DTF_SHARD_MIN_ROWS", "1000")
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd import _native
    from distributed_tensorflow_example_amd.compat import lowering

    real = _native.load()
    monkeypatch.setattr(_native, "load", lambda: _Native(real))
    F, B = 5000, 8
    tf.reset_default_graph()
    with tf.device(tf.train.replica_device_setter(ps_tasks=1)):
        gs = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0), trainable=False)
        shp, ind, fid, fvl = (tf.placeholder(tf.int64), tf.placeholder(tf.int64), tf.placeholder(tf.int64),
                              tf.placeholder(tf.float32))
        y = tf.placeholder(tf.float32, [None, 1])
        W = tf.Variable(tf.random_normal([F, 1]))
        b = tf.Variable(tf.zeros([1]))
        logits = tf.add(tf.nn.embedding_lookup_sparse(W, tf.SparseTensor(shape=shp, indices=ind, values=fid),
                                                      tf.SparseTensor(shape=shp, indices=ind, values=fvl),
                                                      combiner="sum"), b)
        loss = tf.reduce_mean(tf.nn.sigmoid_cross_entropy_with_logits(logits, y))
        train = tf.train.GradientDescentOptimizer(0.5).minimize(loss, global_step=gs)
    rng = np.random.default_rng(0)
    rows = np.repeat(np.arange(B), 3)
    ids = rng.integers(0, F, rows.size).astype(np.int64)
    feed = {y: np.zeros((B, 1), np.float32), shp: [F, B], ind: np.stack([rows, ids], 1), fid: ids,
            fvl: np.ones(ids.size, np.float32)}
    sess = tf.Session()
    sess.run(tf.global_variables_initializer())
    sess.run([train], feed_dict=feed)                 # CPU: the op-by-op / trainer path builds the plan
    plan = lowering.plan_for(train)
    assert plan is not None
    table = plan.pat.W.table
    monkeypatch.setattr(table, "device", _Dev(), raising=False)
    gv = gs.value
    plan._nplan, plan._nplan_gs = None, True

    # first run on the "GPU": the full path's native call, which installs the runner
    monkeypatch.setattr(plan, "_native_run", lambda ctx, opt, gsv, tb: _first(plan, ctx))
    out = sess.run([train, loss], feed_dict=feed)
    assert out[0] is None and len(sess._fast) == 1
    n0 = plan.steps
    for _ in range(3):
        out = sess.run([train, loss], feed_dict=feed)
        assert out[0] is None and float(out[1]) == 0.25
    assert plan.steps == n0 + 3 and len(plan._nplan.calls) == 3
    assert plan._nplan.calls[-1][2] == 0.5
    # a tensor feed: the runner declines, the full path runs
    feed2 = dict(feed)
    feed2[fvl] = torch.ones(ids.size)
    calls = len(plan._nplan.calls)
    sess.run([train, loss], feed_dict=feed2)
    assert len(plan._nplan.calls) == calls
    sess.close()
    tf.reset_default_graph()
    del gv


def _first(plan, ctx):
    if plan._nplan is None:
        plan._nplan = _Plan()
    plan._nplan_gs = True
    ctx.memo[id(plan.pat.loss)] = plan._nplan.loss()
    ctx.memo[id(plan.op)] = None
    plan.steps += 1
    return True
