"""TF sparse-update semantics at the edges of the sharded-table machinery:

* several lookups of one partitioned variable in a step: the IndexedSlices are
  summed and a non-linear rule (Adagrad) is applied ONCE (compat/train.py);
* Adam's beta1_power / beta2_power are saved and a restore resumes the step
  count of the dense and the partitioned (sparse) Adam;
* an empty batch touches no table row (the static padding must not count as a
  touched row under momentum);
* a checkpoint taken mid-window holds the voided-and-not-yet-replayed steps;
* Wide&Deep's checkpoint holds its whole Adam state and restores it.
"""
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
F = 1200


def _two_lookup_graph(tf, opt):
    with tf.device(tf.train.replica_device_setter(ps_tasks=1)):
        gs = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0), trainable=False)
        ph = {}
        for k in ("a", "b"):
            ph[k] = (tf.placeholder(tf.int64), tf.placeholder(tf.int64), tf.placeholder(tf.int64),
                     tf.placeholder(tf.float32))
        y = tf.placeholder(tf.float32, [None, 1])
        with tf.name_scope("weights"):
            W = tf.Variable(tf.random_normal([F, 1]))
        with tf.name_scope("bias"):
            b = tf.Variable(tf.zeros([1]))
        outs = []
        for k in ("a", "b"):
            shp, idx, fid, fv = ph[k]
            outs.append(tf.nn.embedding_lookup_sparse(W, tf.SparseTensor(shape=shp, indices=idx, values=fid),
                                                      tf.SparseTensor(shape=shp, indices=idx, values=fv),
                                                      combiner="sum"))
        py_x = outs[0] + outs[1] + b
        ce = tf.reduce_mean(tf.nn.sigmoid_cross_entropy_with_logits(py_x, y))
        train = opt.minimize(ce, global_step=gs)
    return dict(gs=gs, ph=ph, y=y, W=W, b=b, train=train)


def _csr(rng, B, nnz):
    fids = rng.integers(0, 60, size=(B, nnz)).astype(np.int64)        # small id range: overlap between lookups
    fvals = rng.standard_normal((B, nnz)).astype(np.float32)
    rows = np.repeat(np.arange(B), nnz)
    idx = np.stack([rows, np.tile(np.arange(nnz), B)], 1).astype(np.int64)
    return fids, fvals, idx


def test_two_lookups_of_one_partitioned_variable_apply_adagrad_once(monkeypatch):
    monkeypatch.setenv("DTF_SHARD_MIN_ROWS", "1000")
    import distributed_tensorflow_example_amd.compat as tf

    tf.reset_default_graph()
    tf.set_random_seed(3)
    lr, acc0 = 0.5, 0.1
    g = _two_lookup_graph(tf, tf.train.AdagradOptimizer(lr, initial_accumulator_value=acc0))
    assert type(g["W"]).__name__ == "PartitionedVariable"
    rng = np.random.default_rng(0)
    B, nnz = 16, 5
    fa, va, ia = _csr(rng, B, nnz)
    fb, vb, ib = _csr(rng, B, nnz)
    y = (rng.random((B, 1)) < 0.5).astype(np.float32)
    feed = {g["y"]: y}
    for k, (f, v, i) in (("a", (fa, va, ia)), ("b", (fb, vb, ib))):
        shp, idx, fid, fv = g["ph"][k]
        feed.update({shp: np.array([F, B]), idx: i, fid: f.reshape(-1), fv: v.reshape(-1)})
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        W0 = g["W"].numpy().astype(np.float64).reshape(-1)
        sess.run(g["train"], feed_dict=feed)
        W1 = g["W"].numpy().astype(np.float64).reshape(-1)
    # fp64 reference: summed gradient of both lookups, Adagrad once on the touched rows
    Wt = torch.tensor(W0, requires_grad=True)
    z = (Wt[torch.from_numpy(fa)] * torch.from_numpy(va).double()).sum(1) + \
        (Wt[torch.from_numpy(fb)] * torch.from_numpy(vb).double()).sum(1)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(z, torch.from_numpy(y).double().reshape(-1))
    loss.backward()
    gW = Wt.grad.numpy()
    touched = np.zeros(F, bool)
    touched[fa.reshape(-1)] = True
    touched[fb.reshape(-1)] = True
    want = W0.copy()
    acc = acc0 + gW ** 2
    want[touched] -= lr * gW[touched] / np.sqrt(acc[touched])
    np.testing.assert_allclose(W1, want, rtol=1e-5, atol=1e-6)


def test_adam_powers_restore_dense_and_sparse_step(monkeypatch, tmp_path):
    monkeypatch.setenv("DTF_SHARD_MIN_ROWS", "1000")
    import distributed_tensorflow_example_amd.compat as tf

    rng = np.random.default_rng(1)
    B, nnz = 16, 5
    fa, va, ia = _csr(rng, B, nnz)
    fb, vb, ib = _csr(rng, B, nnz)
    y = (rng.random((B, 1)) < 0.5).astype(np.float32)

    def feed_of(g):
        feed = {g["y"]: y}
        for k, (f, v, i) in (("a", (fa, va, ia)), ("b", (fb, vb, ib))):
            shp, idx, fid, fv = g["ph"][k]
            feed.update({shp: np.array([F, B]), idx: i, fid: f.reshape(-1), fv: v.reshape(-1)})
        return feed

    tf.reset_default_graph()
    tf.set_random_seed(3)
    g = _two_lookup_graph(tf, tf.train.AdamOptimizer(0.01))
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        for _ in range(3):
            sess.run(g["train"], feed_dict=feed_of(g))
        path = tf.train.Saver().save(sess, str(tmp_path / "m"), global_step=g["gs"])
        sess.run(g["train"], feed_dict=feed_of(g))
        w_cont = g["W"].numpy().copy()
        b_cont = sess.run(g["b"]).copy()
    from distributed_tensorflow_example_amd.compat import saver

    assert abs(float(saver.read_tensor(path, "beta1_power")) - 0.9 ** 4) < 1e-6
    tf.reset_default_graph()
    tf.set_random_seed(99)                       # different init: the restore must bring everything back
    g2 = _two_lookup_graph(tf, tf.train.AdamOptimizer(0.01))
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        tf.train.Saver().restore(sess, path)
        assert int(g2["W"].table._adam.step_t.item()) == 3
        sess.run(g2["train"], feed_dict=feed_of(g2))
        np.testing.assert_allclose(g2["W"].numpy(), w_cont, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(sess.run(g2["b"]), b_cont, rtol=1e-6, atol=1e-7)


def test_empty_batch_touches_no_row_under_momentum():
    from distributed_tensorflow_example_amd.models.wide_deep import WideDeep
    from distributed_tensorflow_example_amd.parallel.world import World

    m = WideDeep(500, emb_dim=4, hidden=(8,), lr=0.1, world=World(device="cpu"), device="cpu",
                 ids_capacity=64, rows=4, sparse_opt="momentum", sparse_hp={"momentum": 0.9})
    ids = torch.tensor([0, 3, 0, 7, 9, 3, 0, 11])
    offs = torch.tensor([0, 2, 4, 6, 8])
    m.train_step((torch.ones(4, 1), offs, ids, torch.ones(8)))
    assert float(m.emb.slots["Momentum"][0].abs().sum()) > 0          # row 0 carries momentum
    before = m.emb.local.clone(), m.wide.local.clone()
    m.train_step((torch.zeros(4, 1), torch.zeros(5, dtype=torch.int64), torch.zeros(0, dtype=torch.int64),
                  torch.zeros(0)))
    assert torch.equal(m.emb.local, before[0]) and torch.equal(m.wide.local, before[1])
    # a non-empty batch afterwards moves row 0 again (the flag is per batch)
    m.train_step((torch.ones(4, 1), offs, ids, torch.ones(8)))
    assert not torch.equal(m.emb.local[0], before[0][0])


def test_checkpoint_mid_window_holds_voided_steps(tmp_path):
    """4 ranks, per-peer capacity 1: every step is voided and waits for the
    window's replay; a checkpoint taken before any explicit sync_exchange must
    still equal one rank trained on the whole batch."""
    from distributed_tensorflow_example_amd.compat import saver
    from distributed_tensorflow_example_amd.data import libsvm

    sys.path.insert(0, os.path.join(REPO, "tests"))
    import test_sparse_cpu as T

    files = libsvm.write_synthetic(str(tmp_path / "train" / "part"), 2, 700, 3000, 12, seed=0)
    one = T._run(1, files, 3, 0.5, "lr")
    four = T._run(4, files, 3, 0.5, "lr-static", 1, "sgd", False)
    prefix = four[0][4]
    w_ck = saver.read_tensor(prefix, "weights/Variable").numpy()
    assert np.allclose(w_ck, one[0][2], atol=1e-5)
    assert abs(float(saver.read_tensor(prefix, "bias/Variable")[0]) - one[0][3]) < 1e-6


def test_wide_deep_checkpoint_restores_adam_state(tmp_path):
    from distributed_tensorflow_example_amd import ckpt
    from distributed_tensorflow_example_amd.models.wide_deep import WideDeep
    from distributed_tensorflow_example_amd.parallel.world import World

    def make(seed):
        return WideDeep(400, emb_dim=4, hidden=(8,), lr=0.1, dense_opt="adam", dense_lr=0.01,
                        world=World(device="cpu"), device="cpu", seed=seed, sparse_opt="adam")
    rng = np.random.default_rng(2)

    def batch():
        ids = torch.from_numpy(rng.integers(0, 400, 24)).long()
        return (torch.from_numpy((rng.random((6, 1)) < 0.5).astype(np.float32)),
                torch.arange(0, 25, 4, dtype=torch.int64), ids, torch.ones(24))
    bs = [batch() for _ in range(4)]
    a = make(1)
    for b in bs[:3]:
        a.train_step(b)
    local, repl = a.checkpoint_tensors()
    assert {"beta1_power", "sparse/beta1_power", "deep/dense_0/kernel/Adam_1", "deep/embedding/Adam"} <= \
        set(local) | set(repl)
    prefix = ckpt.save_sharded(str(tmp_path / "wd"), local, repl, World(device="cpu"), global_step=a.global_step)
    a.train_step(bs[3])
    c = make(7)
    c.restore(prefix)
    assert int(c.opt.step_t.item()) == 3 and int(c.wide._adam.step_t.item()) == 3 and c.global_step == 3
    c.train_step(bs[3])
    assert torch.allclose(c.emb.local, a.emb.local, atol=1e-7) and torch.allclose(c.wide.local, a.wide.local, atol=1e-7)
    for p, q in zip(c.dense_params, a.dense_params):
        assert torch.allclose(p, q, atol=1e-7)


def test_adam_steps_from_powers_survives_underflow():
    """beta1 = 0.9 underflows float32 near t = 990 and beta2 = 0.999 near
    t ~ 103k: the count comes from whichever power is still normal, and a fully
    underflowed pair saturates (bias correction 1) instead of restarting at 0."""
    from distributed_tensorflow_example_amd.optim import adam_steps_from_powers

    def f32(x):
        return float(np.float32(x))

    for t in (0, 3, 500, 829, 900, 990, 1200, 5000, 60000):
        b1, b2 = f32(0.9 ** (t + 1)), f32(0.999 ** (t + 1))
        assert adam_steps_from_powers(b1, 0.9, b2, 0.999) == t
        assert adam_steps_from_powers(b2, 0.999, b1, 0.9) == t
    # beta1's power alone, still normal
    assert adam_steps_from_powers(f32(0.9 ** 501), 0.9) == 500
    # beta1's alone once it underflowed: a lower bound past the underflow, never 0
    assert adam_steps_from_powers(0.0, 0.9) >= 986
    # both underflowed: saturated at a count where both float32 powers are 0
    t = adam_steps_from_powers(0.0, 0.9, 0.0, 0.999)
    assert f32(0.9 ** (t + 1)) == 0.0 and f32(0.999 ** (t + 1)) == 0.0


def test_wide_deep_restore_after_1000_adam_steps(tmp_path):
    from distributed_tensorflow_example_amd import ckpt
    from distributed_tensorflow_example_amd.models.wide_deep import WideDeep
    from distributed_tensorflow_example_amd.parallel.world import World

    def make(seed):
        return WideDeep(400, emb_dim=4, hidden=(8,), lr=0.1, dense_opt="adam", dense_lr=0.01,
                        world=World(device="cpu"), device="cpu", seed=seed, sparse_opt="adam")
    a = make(1)
    for o in (a.opt, a.wide._adam, a.emb._adam):
        o.step_t.fill_(1234)          # past beta1_power's float32 underflow
    local, repl = a.checkpoint_tensors()
    assert float(repl["beta1_power"]) == 0.0 and int(repl["adam_step"]) == 1234
    prefix = ckpt.save_sharded(str(tmp_path / "wd"), local, repl, World(device="cpu"), global_step=1234)
    c = make(7)
    c.restore(prefix)
    assert int(c.opt.step_t.item()) == 1234 and int(c.wide._adam.step_t.item()) == 1234
    assert int(c.emb._adam.step_t.item()) == 1234


def test_compat_power_restore_any_order_past_underflow():
    """Saver.restore feeds beta1_power / beta2_power one at a time: the tied
    step count must come out right in either order once beta1's power is 0."""
    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat.train import _PowerVariable

    for order in ((0, 1), (1, 0)):
        step = torch.zeros(1, dtype=torch.int64)
        p1, p2 = _PowerVariable("beta1_power", 0.9, [step]), _PowerVariable("beta2_power", 0.999, [step])
        p1.sibling, p2.sibling = p2, p1
        vals = (torch.tensor(np.float32(0.9 ** 2001)), torch.tensor(np.float32(0.999 ** 2001)))
        assert float(vals[0]) == 0.0
        pv = (p1, p2)
        for i in order:
            pv[i].restore_from(vals[i])
        assert int(step.item()) == 2000, order
    assert tf is not None
