"""Pattern matching of the compat graph lowering (compat/lowering.py) on CPU:
the reference training graph (example.py:93-118) is recognised in its naive
and stable forms, the accuracy node is found, fetch sets that read matched
interior nodes are refused, and CPU sessions never lower."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _graph(tf, stable=False, act="sigmoid", opt="sgd"):
    tf.reset_default_graph()
    gs = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0), trainable=False)
    x = tf.placeholder(tf.float32, [None, 784], name="x-input")
    y_ = tf.placeholder(tf.float32, [None, 10], name="y-input")
    W1 = tf.Variable(tf.random_normal([784, 100], seed=1))
    W2 = tf.Variable(tf.random_normal([100, 10], seed=2))
    b1 = tf.Variable(tf.zeros([100]))
    b2 = tf.Variable(tf.zeros([10]))
    a2 = (tf.nn.sigmoid if act == "sigmoid" else tf.nn.relu)(tf.add(tf.matmul(x, W1), b1))
    z3 = tf.add(tf.matmul(a2, W2), b2)
    y = tf.nn.softmax(z3)
    if stable:
        ce = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(labels=y_, logits=z3))
    else:
        ce = tf.reduce_mean(-tf.reduce_sum(y_ * tf.log(y), reduction_indices=[1]))
    o = {"sgd": lambda: tf.train.GradientDescentOptimizer(0.5), "adam": lambda: tf.train.AdamOptimizer(0.01),
         "momentum": lambda: tf.train.MomentumOptimizer(0.1, 0.9)}[opt]()
    train = o.minimize(ce, global_step=gs)
    acc = tf.reduce_mean(tf.cast(tf.equal(tf.argmax(y, 1), tf.argmax(y_, 1)), tf.float32))
    return dict(x=x, y_=y_, W=[W1, W2, b1, b2], y=y, ce=ce, train=train, acc=acc, gs=gs, a2=a2)


def test_match_reference_graph_forms():
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L

    for stable in (False, True):
        for act in ("sigmoid", "relu"):
            g = _graph(tf, stable, act)
            p = L.match_mlp(g["ce"])
            assert p is not None and p.naive == (not stable) and p.act == (0 if act == "sigmoid" else 1)
            assert [p.W1, p.W2, p.b1, p.b2] == g["W"] and p.x is g["x"] and p.ylab is g["y_"]
            plan = L.MLPStepPlan(g["train"], p, tf.get_default_graph())
            assert plan.accuracy is g["acc"]
            assert plan.fetches_ok([g["train"], g["ce"], g["acc"], g["gs"]])
            assert not plan.fetches_ok([g["train"], g["y"]])          # would read post-update weights
            assert not plan.fetches_ok([g["train"], g["W"][0]])
    tf.reset_default_graph()


def test_no_match_for_other_graphs():
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L

    tf.reset_default_graph()
    x = tf.placeholder(tf.float32, [None, 4])
    W = tf.Variable(tf.zeros([4, 3]))
    b = tf.Variable(tf.zeros([3]))
    y = tf.nn.softmax(tf.matmul(x, W) + b)                 # single layer: not the MLP pattern
    y_ = tf.placeholder(tf.float32, [None, 3])
    ce = tf.reduce_mean(-tf.reduce_sum(y_ * tf.log(y), reduction_indices=[1]))
    assert L.match_mlp(ce) is None
    ce2 = tf.reduce_mean(-tf.reduce_sum(y_ * tf.log(y), reduction_indices=[0]))
    assert L.match_mlp(ce2) is None
    tf.reset_default_graph()


def test_cpu_session_runs_eagerly():
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L

    g = _graph(tf)
    rng = np.random.default_rng(0)
    bx = rng.random((20, 784), dtype=np.float32)
    by = np.eye(10, dtype=np.float32)[rng.integers(0, 10, 20)]
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        _, c = sess.run([g["train"], g["ce"]], feed_dict={g["x"]: bx, g["y_"]: by})
        assert np.isfinite(c)
    import torch

    if not torch.cuda.is_available():
        assert L.plan_for(g["train"]) is None               # CPU sessions never lower
    tf.reset_default_graph()


def test_auc_update_on_the_model_blocks_lowering():
    """streaming_auc keeps its graph edges (predictions, labels, confusion
    variables): a run fetching [train_op, auc_update] on the MLP pattern reads
    the weights the fused step updates, so it must not be lowered (the AUC would
    see post-update weights)."""
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering as L

    g = _graph(tf)
    p = L.match_mlp(g["ce"])
    plan = L.MLPStepPlan(g["train"], p, tf.get_default_graph())
    auc_val, auc_upd = tf.contrib.metrics.streaming_auc(g["y"][:, 1], g["y_"][:, 1])
    assert len(auc_upd.inputs) == 6 and len(auc_val.inputs) == 4      # preds, labels + tp, fn, tn, fp
    assert not plan.fetches_ok([g["train"], auc_upd])
    assert plan.fetches_ok([g["train"], g["ce"]])
    tf.reset_default_graph()
