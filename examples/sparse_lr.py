"""Sparse logistic regression over libsvm shards -- counterpart of lr2.py.

    python examples/sparse_lr.py --job_name=ps     --task_index=0 --cluster_conf=cluster_conf.json ...
    python examples/sparse_lr.py --job_name=worker --task_index=0 --cluster_conf=cluster_conf.json \
        --train=hdfs://nn/lr/train/part-* --test=hdfs://nn/lr/test/part-00000 --features=4762348

Same flags and console lines as the reference (lr2.py:19-35, :307-315,
:447-468).  Differences (see README):
* W[F,1] is row-sharded across the workers' GPUs (ps role, all-to-all
  lookups/updates) instead of living on ps0; b is replicated;
* training is synchronous; each epoch runs min-over-workers batches so every
  rank issues the same collectives;
* the final AUC aggregates every worker's test shard (all-reduced
  histograms), not one worker's view;
* `--mode=queue` uses the native looping LibsvmStream (C++ threads), with
  `--steps_per_epoch` bounding an epoch (the reference loops forever);
* `--checkpoint` writes a sharded TF V2 bundle at the end (lr2.py only
  declares the flag).
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import distributed_tensorflow_example_amd.compat as tf  # noqa: E402
from distributed_tensorflow_example_amd import ckpt  # noqa: E402
from distributed_tensorflow_example_amd.data import libsvm  # noqa: E402
from distributed_tensorflow_example_amd.models import sparse_lr  # noqa: E402
from distributed_tensorflow_example_amd.utils.logging import TaskLogger  # noqa: E402

flags = tf.app.flags
flags.DEFINE_string("job_name", "worker", "job name")
flags.DEFINE_integer("task_index", 0, "task index")
flags.DEFINE_integer("thread_num", 2, "parser threads")
flags.DEFINE_float("learning_rate", 0.001, "Initial learning rate.")
flags.DEFINE_integer("num_epochs", 120, "Number of epochs to run trainer.")
flags.DEFINE_integer("batch_size", 500, "Batch size.")
flags.DEFINE_integer("features", 4762348, "Feature size")
flags.DEFINE_string("train", "", "train files: comma list, glob, or @listfile (hdfs:// ok)")
flags.DEFINE_string("test", "", "test files")
flags.DEFINE_string("checkpoint", "", "checkpoint prefix written at the end ('' = none)")
flags.DEFINE_integer("trace_step_interval", 10000, "number of steps to output info")
flags.DEFINE_float("train_sampling_rate", 1.0, "sampling rate for train file")
flags.DEFINE_float("test_sampling_rate", 1.0, "sampling rate for test file")
flags.DEFINE_string("mode", "all", "load data all or queue")
flags.DEFINE_integer("train_queue_capacity", 2000, "train queue capacity (samples)")
flags.DEFINE_integer("test_queue_capacity", 2000, "test queue capacity (samples)")
flags.DEFINE_integer("steps_per_epoch", 100, "queue mode: batches per epoch")
flags.DEFINE_string("cluster_conf", "cluster_conf.json", "cluster JSON (lr2.py:325)")
flags.DEFINE_integer("seed", 1, "init seed")
flags.DEFINE_string("result_json", "", "write final metrics here (tests)")
flags.DEFINE_string("update_mode", "", "sync (default: all-reduce / sharded exchange per step) or async (the "
                    "reference's Hogwild ps updates: rows read from and scattered into the owners' shared shards); "
                    "'' = $DTF_UPDATE_MODE or sync")
flags.DEFINE_boolean("use_locking", False, "async: no lost updates (CAS / file locks), TF's use_locking")
FLAGS = flags.FLAGS


def main(_argv):
    with open(FLAGS.cluster_conf) as f:
        cluster = tf.train.ClusterSpec(json.load(f))
    num_workers = cluster.num_tasks("worker")
    log = TaskLogger(FLAGS.job_name, FLAGS.task_index)
    server = tf.train.Server(cluster, job_name=FLAGS.job_name, task_index=FLAGS.task_index)
    if FLAGS.job_name == "ps":
        log.info("start ...")
        server.join()
        log.info("Terminating parameter server")
        return 0

    log.info("start ...")
    world = server.world
    dp = libsvm.DataProvider(num_workers, FLAGS.task_index, FLAGS.thread_num, FLAGS.mode, train=FLAGS.train,
                             test=FLAGS.test, batch_size=FLAGS.batch_size,
                             train_sampling_rate=FLAGS.train_sampling_rate,
                             test_sampling_rate=FLAGS.test_sampling_rate,
                             queue_capacity=max(2, FLAGS.train_queue_capacity // FLAGS.batch_size),
                             seed=FLAGS.seed).init()
    log.info("load data")
    dp.LoadData()
    log.info("build model")
    model = sparse_lr.SparseLRTrainer(FLAGS.features, FLAGS.learning_rate, world, seed=FLAGS.seed,
                                      update_mode=FLAGS.update_mode or None, use_locking=FLAGS.use_locking)
    log.info("sampling test data ...")
    test_data = dp.GetTestSamplesSampled(sampling_rate=0.1, sampling_max_num=1000)

    def test(epoch, step):
        loss, _ = model.evaluate(test_data)
        loss = world.host_all_reduce(float(loss)) / world.world_size
        log.info(f"epoch: {epoch}, local step: {step}, global step: {model.global_step}, loss: {loss}")
        return loss

    log.info("Start train ...")
    t0 = time.time()
    step = 0
    last_loss = None
    for epoch in range(FLAGS.num_epochs):
        dp.Shuffle()
        if FLAGS.mode == "all":
            nb = sparse_lr.steps_per_epoch(world, -(-len(dp.GetTrainSamples()) // FLAGS.batch_size))
        else:
            nb = FLAGS.steps_per_epoch
        for batch in dp.NextBatch("train", max_batches=nb):
            model.train_step(batch)
            step += 1
            if step % FLAGS.trace_step_interval == 0:
                test(epoch, step)
        last_loss = test(epoch, step)
    train_s = time.time() - t0
    log.info(f"Finish train. {step} steps in {train_s:.2f}s")

    log.info("Start evaluate ...")
    model.reset_auc()
    nt = -(-len(dp.GetTestSamples()) // FLAGS.batch_size) if FLAGS.mode == "all" else 10
    nt = sparse_lr.steps_per_epoch(world, nt)
    for batch in dp.NextBatch("test", max_batches=nt):
        model.auc_update(batch)
    auc = model.auc(all_workers=True)       # (a collective: every worker finished training)
    model.refresh_global_step()
    log.info(f"Finish evaluate, auc: {auc}")
    if FLAGS.checkpoint:
        local, repl = model.checkpoint_tensors()
        path = ckpt.save_sharded(FLAGS.checkpoint, local, repl, world, global_step=model.global_step)
        log.info(f"saved checkpoint {path}")
    if FLAGS.result_json:
        with open(FLAGS.result_json, "w") as f:
            json.dump({"auc": auc, "loss": last_loss, "global_step": model.global_step,
                       "b": float(model.b.detach().cpu()[0]), "steps": step, "train_s": train_s}, f)
    dp.close()
    server.signal_done()
    return 0


if __name__ == "__main__":
    tf.app.run(main)
