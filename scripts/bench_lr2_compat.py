#!/usr/bin/env python3
"""lr2.py's train run through the compat Session (examples/lr2_compat.py's
graph: replica_device_setter, SparseTensor feeds, embedding_lookup_sparse,
sigmoid xent, GradientDescentOptimizer) vs the native SparseLRTrainer step on
the same data -- the lowered Session.run (compat/lowering.py SparseLRStepPlan)
vs the native step on device-resident batches and on the same host (numpy)
batches the Session is fed.

    python scripts/bench_lr2_compat.py [--features 1e9] [--batch 500] [--nnz 40] [--steps 200]

Synthetic libsvm-shaped batches (Zipf-1.1 ids, like scripts/bench_models.py);
feeds are built before the timed loop (the reference builds them in Python,
lr2.py:439, which is not the Session's cost).  One JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def batches(n, B, F, nnz, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k = rng.integers(nnz // 2, nnz + nnz // 2 + 1, size=B)          # ragged rows, like libsvm lines
        offs = np.zeros(B + 1, np.int64)
        np.cumsum(k, out=offs[1:])
        ids = ((rng.zipf(1.1, int(offs[-1])) - 1) % F).astype(np.int64)
        vals = rng.random(int(offs[-1])).astype(np.float32)
        lab = (rng.random((B, 1)) < 0.3).astype(np.float32)
        out.append((lab, offs, ids, vals))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--features", type=float, default=1e9)
    ap.add_argument("--batch", type=int, default=500)
    ap.add_argument("--nnz", type=int, default=40)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--lr", type=float, default=1.0)
    a = ap.parse_args()
    F = int(a.features)
    import torch

    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.compat import lowering
    from distributed_tensorflow_example_amd.models.sparse_lr import SparseLRTrainer
    from distributed_tensorflow_example_amd.parallel.world import World

    dev = torch.device("cuda", 0)
    data = batches(16, a.batch, F, a.nnz, 1234)
    with tf.device(tf.train.replica_device_setter(ps_tasks=1)):
        global_step = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0), trainable=False)
        x_shape = tf.placeholder(tf.int64)
        x_indices = tf.placeholder(tf.int64)
        x_fids = tf.placeholder(tf.int64)
        x_fvals = tf.placeholder(tf.float32)
        sp_fids = tf.SparseTensor(shape=x_shape, indices=x_indices, values=x_fids)
        sp_fvals = tf.SparseTensor(shape=x_shape, indices=x_indices, values=x_fvals)
        y = tf.placeholder(tf.float32, [None, 1])
        with tf.name_scope("weights"):
            W = tf.Variable(tf.random_normal([F, 1]))
        with tf.name_scope("bias"):
            b = tf.Variable(tf.zeros([1]))
        py_x = tf.add(tf.nn.embedding_lookup_sparse(W, sp_fids, sp_fvals, combiner="sum"), b)
        cross_entropy = tf.reduce_mean(tf.nn.sigmoid_cross_entropy_with_logits(py_x, y))
        train_op = tf.train.GradientDescentOptimizer(a.lr).minimize(cross_entropy, global_step=global_step)
    feeds = []
    for lab, offs, ids, vals in data:
        rows = np.repeat(np.arange(a.batch, dtype=np.int64), np.diff(offs))
        feeds.append({y: lab, x_shape: [F, a.batch], x_indices: np.stack([rows, ids], 1), x_fids: ids,
                      x_fvals: vals})
    sess = tf.Session()
    sess.run(tf.global_variables_initializer())
    for i in range(a.warmup):
        sess.run([train_op], feed_dict=feeds[i % 16])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        sess.run([train_op], feed_dict=feeds[i % 16])
    torch.cuda.synchronize()
    sess_ms = (time.perf_counter() - t0) / a.steps * 1e3
    plan = lowering.plan_for(train_op)
    lowered = plan.steps if plan is not None else 0
    nplan = getattr(plan, "_nplan", None) if plan is not None else None
    native_split = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in nplan.timing().items()} \
        if nplan is not None else None
    loss_c = float(sess.run(cross_entropy, feed_dict=feeds[0]))
    del sess

    tr = SparseLRTrainer(F, a.lr, World(device=dev), device=dev)
    tr.enable_graph()
    dev_batches = []
    for lab, offs, ids, vals in data:    # native: batches padded like the lowered plan's id buckets
        n = ids.size
        cap = -(-n // 4096) * 4096
        ids_p = np.concatenate([ids, np.full(cap - n, ids[0])])
        vals_p = np.concatenate([vals, np.zeros(cap - n, np.float32)])
        offs_p = offs.copy()
        offs_p[-1] = cap
        dev_batches.append(tuple(torch.from_numpy(x).to(dev) for x in (lab, offs_p, ids_p, vals_p)))
    for i in range(a.warmup):
        tr.train_step(dev_batches[i % 16])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        tr.train_step(dev_batches[i % 16])
    torch.cuda.synchronize()
    nat_ms = (time.perf_counter() - t0) / a.steps * 1e3
    # native, host-fed: the same numpy CSR batches each step (the compat Session's
    # situation -- its feeds are host arrays): SparseLRPlan.run_csr
    for i in range(a.warmup):
        tr.train_step(data[i % 16])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        tr.train_step(data[i % 16])
    torch.cuda.synchronize()
    host_ms = (time.perf_counter() - t0) / a.steps * 1e3
    host_split = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in tr._plan.timing().items()}
    print(json.dumps({"metric": "lr2 compat Session.run vs native sparse-LR step (ms)", "features": F,
                      "batch": a.batch, "nnz_per_sample": a.nnz, "steps": a.steps,
                      "session_run_ms": round(sess_ms, 4),
                      # the Session's compat overhead: the native trainer fed the SAME host (numpy)
                      # batches every step, as the Session is (lr2.py's feed_dict)
                      "native_host_fed_step_ms": round(host_ms, 4),
                      "ratio": round(sess_ms / host_ms, 3),
                      "ratio_basis": "native SparseLRTrainer step on the same host numpy batches",
                      # and against a native step whose batches already sit on the GPU (no host feed at all)
                      "native_device_batches_step_ms": round(nat_ms, 4),
                      "ratio_vs_device_resident_batches": round(sess_ms / nat_ms, 3),
                      "native_host_fed_split_us": host_split,
                      "lowered_runs": lowered,
                      "session_samples_per_s": round(a.batch / sess_ms * 1e3, 1),
                      "session_native_call_split_us": native_split,
                      "native_host_fed_samples_per_s": round(a.batch / host_ms * 1e3, 1),
                      "loss_after_compat_run": round(loss_c, 5)}), flush=True)


if __name__ == "__main__":
    main()
