"""lr2.py as written, through the TF-1.x compat API (reference: lr2.py:318-476).

    python examples/lr2_compat.py --job_name=ps     --task_index=0 --cluster_conf=cluster_conf.json ...
    python examples/lr2_compat.py --job_name=worker --task_index=0 --cluster_conf=cluster_conf.json \
        --train=hdfs://nn/lr/train/part-* --test=hdfs://nn/lr/test/part-00000 --features=4762348

The graph is built the way the reference builds it -- `replica_device_setter`,
placeholders fed as a SparseTensor, `embedding_lookup_sparse(W, ...,
combiner='sum') + b`, `sigmoid_cross_entropy_with_logits`,
`GradientDescentOptimizer.minimize(loss, global_step)`, `streaming_auc`,
`Supervisor.prepare_or_wait_for_session` -- and trained with
`sess.run([train_op], feed_dict={y, x_shape, x_indices, x_fids, x_fvals})`.
On this runtime the ps-placed W[F, 1] is a row-sharded PartitionedVariable
(one shard per worker GPU) and the Session lowers the train run onto the
native sparse-LR step (compat/lowering.py; DTF_GRAPH_LOWERING=0 runs it op by
op).  examples/sparse_lr.py is the same program on the native API.
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import distributed_tensorflow_example_amd.compat as tf  # noqa: E402
from distributed_tensorflow_example_amd.data.libsvm import DataProvider  # noqa: E402
from distributed_tensorflow_example_amd.utils.logging import TaskLogger  # noqa: E402

flags = tf.app.flags
flags.DEFINE_string("job_name", "worker", "job name: worker or ps")
flags.DEFINE_integer("task_index", 0, "Worker task index, should be >= 0. task_index=0 is the chief worker task")
flags.DEFINE_integer("thread_num", 2, "Number of reading threads")
flags.DEFINE_float("learning_rate", 0.001, "Initial learning rate.")
flags.DEFINE_integer("num_epochs", 120, "Number of epochs to run trainer.")
flags.DEFINE_integer("batch_size", 500, "Batch size.")
flags.DEFINE_integer("features", 4762348, "Feature size")
flags.DEFINE_string("train", "", "train files: comma list, glob, or @listfile (hdfs:// ok)")
flags.DEFINE_string("test", "", "test files")
flags.DEFINE_integer("trace_step_interval", 10000, "number of steps to output info")
flags.DEFINE_float("train_sampling_rate", 1.0, "sampling rate for train file")
flags.DEFINE_float("test_sampling_rate", 1.0, "sampling rate for test file")
flags.DEFINE_string("mode", "all", "load data all or queue")
flags.DEFINE_string("cluster_conf", "cluster_conf.json", "cluster JSON (lr2.py:325)")
flags.DEFINE_string("result_json", "", "write final metrics here (tests)")
FLAGS = flags.FLAGS


def main(_):
    learning_rate = FLAGS.learning_rate
    num_epochs = FLAGS.num_epochs
    num_features = FLAGS.features
    trace_step_interval = FLAGS.trace_step_interval
    log = TaskLogger(FLAGS.job_name, FLAGS.task_index)

    cluster_conf = json.load(open(FLAGS.cluster_conf, "r"))
    cluster_spec = tf.train.ClusterSpec(cluster_conf)
    num_workers = len(cluster_conf["worker"])
    server = tf.train.Server(cluster_spec, job_name=FLAGS.job_name, task_index=FLAGS.task_index)
    if FLAGS.job_name == "ps":
        log.info("start ...")
        server.join()
        return 0

    log.info("start ...")
    is_chief = FLAGS.task_index == 0
    data_provider = DataProvider(num_workers, FLAGS.task_index, FLAGS.thread_num, FLAGS.mode, train=FLAGS.train,
                                 test=FLAGS.test, batch_size=FLAGS.batch_size,
                                 train_sampling_rate=FLAGS.train_sampling_rate,
                                 test_sampling_rate=FLAGS.test_sampling_rate)
    data_provider.init()
    log.info("load data")
    data_provider.LoadData()

    log.info("build graph")
    with tf.device(tf.train.replica_device_setter(worker_device="/job:worker/task:%d" % FLAGS.task_index,
                                                  cluster=cluster_spec)):
        global_step = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0), trainable=False)
        with tf.name_scope("input"):
            x_shape = tf.placeholder(tf.int64)
            x_indices = tf.placeholder(tf.int64)
            x_fids = tf.placeholder(tf.int64)
            x_fvals = tf.placeholder(tf.float32)
            sp_fids = tf.SparseTensor(shape=x_shape, indices=x_indices, values=x_fids)
            sp_fvals = tf.SparseTensor(shape=x_shape, indices=x_indices, values=x_fvals)
            y = tf.placeholder(tf.float32, [None, 1])
        with tf.name_scope("weights"):
            W = tf.Variable(tf.random_normal([num_features, 1]))
        with tf.name_scope("bias"):
            b = tf.Variable(tf.zeros([1]))
        with tf.name_scope("loss"):
            py_x = tf.add(tf.nn.embedding_lookup_sparse(W, sp_fids, sp_fvals, combiner="sum"), b)
            cross_entropy = tf.reduce_mean(tf.nn.sigmoid_cross_entropy_with_logits(py_x, y))
        with tf.name_scope("train"):
            grad_op = tf.train.GradientDescentOptimizer(learning_rate)
            train_op = grad_op.minimize(cross_entropy, global_step=global_step)
        with tf.name_scope("evaluate"):
            predict_op = tf.nn.sigmoid(py_x)
            auc_op = tf.contrib.metrics.streaming_auc(predict_op, y)
        init = [tf.global_variables_initializer(), tf.local_variables_initializer()]
        init_op = tf.global_variables_initializer()
        supervisor = tf.train.Supervisor(is_chief=is_chief, init_op=init, global_step=global_step)
        config = tf.ConfigProto(allow_soft_placement=True)

    # tests: this worker feeds its COO entries in reverse (non-canonical) order
    permute = os.environ.get("DTF_LR2_PERMUTE_COO_TASK") == str(FLAGS.task_index)
    # tests: every worker feeds torch tensors (the lowered step takes numpy feeds;
    # all ranks then run op by op together)
    tensor_feeds = os.environ.get("DTF_LR2_TENSOR_FEEDS") == "1"

    def feed(batch):
        labels, fids, fvals, sp_indices, batch_size = batch.as_tf_feed()
        if permute:
            fids, fvals, sp_indices = fids[::-1], fvals[::-1], sp_indices[::-1]
        if tensor_feeds:
            import torch
            labels, fids, fvals, sp_indices = (torch.from_numpy(np.ascontiguousarray(a))
                                               for a in (labels, fids, fvals, sp_indices))
        return {y: labels, x_shape: [num_features, batch_size], x_indices: sp_indices, x_fids: fids,
                x_fvals: fvals}

    def test(sess, iter_num, step_num, test_data):
        global_step_val, cross_entropy_val = sess.run([global_step, cross_entropy], feed_dict=feed(test_data))
        log.info("epoch: {}, local step: {}, global step: {}, loss: {}".format(
            iter_num, step_num, global_step_val, cross_entropy_val))
        return float(cross_entropy_val)

    log.info("Start session ...")
    with supervisor.prepare_or_wait_for_session(server.target, config=config) as sess:
        sess.run(init_op)      # lr2.py:419 (every worker; chief init + identical seeded values here)
        log.info("sampling test data ...")
        test_data = data_provider.GetTestSamplesSampled(sampling_rate=0.1, sampling_max_num=1000)
        log.info("Start train ...")
        t0 = time.time()
        step_num = 0
        iter_num = 0
        last = None
        # synchronous workers run the same number of steps per epoch (min over workers)
        nb = -(-len(data_provider.GetTrainSamples()) // FLAGS.batch_size)
        if server.world.world_size > 1:
            nb = int(-server.world.host_all_reduce(-float(nb), "max"))
        while iter_num < num_epochs:
            data_provider.Shuffle()
            for batch_samples in data_provider.NextBatch(data_type="train", max_batches=nb):
                if batch_samples is None or batch_samples.size <= 0:
                    break
                sess.run([train_op], feed_dict=feed(batch_samples))
                step_num += 1
                if step_num % trace_step_interval == 0:
                    last = test(sess, iter_num, step_num, test_data)
            last = test(sess, iter_num, step_num, test_data)
            iter_num += 1
        train_s = time.time() - t0
        log.info("Finish train.")

        log.info("Start evaluate ...")
        auc_val = None
        nt = -(-len(data_provider.GetTestSamples()) // FLAGS.batch_size)
        if server.world.world_size > 1:
            nt = int(-server.world.host_all_reduce(-float(nt), "max"))
        for batch_samples in data_provider.NextBatch(data_type="test", max_batches=nt):
            if batch_samples is None or batch_samples.size <= 0:
                break
            auc_val = sess.run(auc_op, feed_dict=feed(batch_samples))
        log.info("Finish evaluate, auc: {}".format(auc_val))
        gstep = float(sess.run(global_step))
        w_final = W.numpy().reshape(-1) if FLAGS.result_json else None
        b_final = float(np.asarray(sess.run(b)).reshape(-1)[0])
    from distributed_tensorflow_example_amd.compat import lowering

    plan = lowering.plan_for(train_op)
    if FLAGS.result_json:
        np.save(FLAGS.result_json + ".W.npy", w_final)
        with open(FLAGS.result_json, "w") as f:
            json.dump({"auc": [float(np.asarray(v).reshape(-1)[0]) for v in auc_val] if auc_val is not None else None,
                       "loss": last, "global_step": gstep, "b": b_final, "steps": step_num, "train_s": train_s,
                       "lowered_steps": plan.steps if plan is not None else 0}, f)
    data_provider.close()
    server.signal_done()
    return 0


if __name__ == "__main__":
    tf.app.run(main=main)
