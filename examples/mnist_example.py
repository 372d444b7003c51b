"""MNIST 784-100-10 sigmoid MLP, ps/worker cluster, written against the TF-1.x
compat front end -- the counterpart of the reference's headline script
(example.py:1-192).

    python examples/mnist_example.py --job_name=ps     --task_index=0
    python examples/mnist_example.py --job_name=worker --task_index=0
    python examples/mnist_example.py --job_name=worker --task_index=1

Cluster: `--ps_hosts/--worker_hosts` (comma lists) or `--cluster_conf` JSON
(cluster_conf.json shape); defaults mirror example.py:23-30 on localhost.

What differs from the reference (README "semantics"):
* workers train *synchronously* by default: every train_op run averages the
  gradients of all workers (on one MI355X node the IPC data plane: the lowered
  step's last kernel all-reduces over xGMI and applies SGD; gloo on CPU) -- the
  SyncReplicasOptimizer path the reference left commented out
  (example.py:109-123); global_step counts sync steps.  `--update_mode=async`
  runs the reference's own asynchronous rule instead (Hogwild updates of shared
  variables, global_step counts every worker's step);
* chief initialises and broadcasts (no re-init race); ps tasks exit from
  `server.join()` once every worker has finished;
* input is the synthetic MNIST-shaped set (no network): same shapes/dtypes;
* `--fused` runs the whole step (fwd+bwd+all-reduce+SGD) as the MFMA
  kernel chain of models.mlp.FusedMLPTrainer instead of the op-by-op graph.
"""
from __future__ import annotations

import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import distributed_tensorflow_example_amd.compat as tf  # noqa: E402
from distributed_tensorflow_example_amd.data import mnist as mnist_data  # noqa: E402
from distributed_tensorflow_example_amd.utils.logging import step_line  # noqa: E402
from distributed_tensorflow_example_amd.utils.metrics import MetricsWriter  # noqa: E402

flags = tf.app.flags
flags.DEFINE_string("job_name", "", "Either 'ps' or 'worker'")
flags.DEFINE_integer("task_index", 0, "Index of task within the job")
flags.DEFINE_string("ps_hosts", "localhost:2222", "comma-separated ps host:port list")
flags.DEFINE_string("worker_hosts", "localhost:2223,localhost:2224", "comma-separated worker host:port list")
flags.DEFINE_string("cluster_conf", "", "JSON file {\"ps\": [...], \"worker\": [...]} (overrides *_hosts)")
flags.DEFINE_integer("batch_size", 100, "per-worker batch")
flags.DEFINE_float("learning_rate", 0.0005, "SGD learning rate")
flags.DEFINE_integer("training_epochs", 5, "epochs over the training split")
flags.DEFINE_integer("max_steps", 0, "stop after this many steps (0 = full epochs)")
flags.DEFINE_integer("train_size", 55000, "synthetic training examples (when no IDX files are found)")
flags.DEFINE_string("data_dir", "", "MNIST IDX directory (train-images-idx3-ubyte[.gz], ...); default "
                    "MNIST_data/{job}_{task} as example.py:60-62; synthetic data if the files are absent")
flags.DEFINE_integer("frequency", 100, "print every N batches")
flags.DEFINE_string("logs_path", "./logs/mnist", "summary root; task dir {job}_{task} appended")
flags.DEFINE_string("activation", "sigmoid", "sigmoid | relu")
flags.DEFINE_boolean("fused", False, "run the fused MFMA train step (GPU only)")
flags.DEFINE_boolean("persistent", False, "with --fused: the persistent weight-stationary engine (one kernel "
                     "launch per epoch, batch <= 112, input streamed from pinned host memory in-kernel)")
flags.DEFINE_string("result_json", "", "write final metrics + params checksum here (tests)")
flags.DEFINE_string("checkpoint_dir", "", "Supervisor logdir: restore on start, checkpoint while training")
flags.DEFINE_integer("save_model_secs", 600, "checkpoint period (chief, seconds)")
flags.DEFINE_integer("save_model_steps", 0, "checkpoint every N global steps (all ranks agree; overrides secs)")
flags.DEFINE_string("metrics_jsonl", "", "append JSON-lines step metrics here")
flags.DEFINE_string("dump_dir", "", "tests: save this worker's initial / final parameters and the batches it fed "
                    "(worker_<task>.npz) and the data-plane facts (which step ran, which collectives)")
flags.DEFINE_string("update_mode", "sync", "sync: every train_op run all-reduces the workers' gradients (default); "
                    "async: the reference's Hogwild ps updates -- each worker applies its own gradient to the "
                    "shared variables without waiting (parallel/async_ps.py), global_step counts every worker's step")
FLAGS = flags.FLAGS


def cluster_spec():
    if FLAGS.cluster_conf:
        with open(FLAGS.cluster_conf) as f:
            return tf.train.ClusterSpec(json.load(f))
    return tf.train.ClusterSpec({"ps": [h for h in FLAGS.ps_hosts.split(",") if h],
                                 "worker": [h for h in FLAGS.worker_hosts.split(",") if h]})


def build_graph(cluster, task_index):
    """Graph of example.py:64-135 (placement, model, loss, SGD, accuracy, summaries)."""
    tf.set_random_seed(1)
    with tf.device(tf.train.replica_device_setter(worker_device=f"/job:worker/task:{task_index}",
                                                  cluster=cluster)):
        global_step = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0),
                                      trainable=False)
        with tf.name_scope("input"):
            x = tf.placeholder(tf.float32, shape=[None, 784], name="x-input")
            y_ = tf.placeholder(tf.float32, shape=[None, 10], name="y-input")
        with tf.name_scope("weights"):
            W1 = tf.Variable(tf.random_normal([784, 100]))
            W2 = tf.Variable(tf.random_normal([100, 10]))
        with tf.name_scope("biases"):
            b1 = tf.Variable(tf.zeros([100]))
            b2 = tf.Variable(tf.zeros([10]))
        with tf.name_scope("softmax"):
            act = tf.nn.sigmoid if FLAGS.activation == "sigmoid" else tf.nn.relu
            a2 = act(tf.add(tf.matmul(x, W1), b1))
            y = tf.nn.softmax(tf.add(tf.matmul(a2, W2), b2))
        with tf.name_scope("cross_entropy"):
            cross_entropy = tf.reduce_mean(-tf.reduce_sum(y_ * tf.log(y), reduction_indices=[1]))
        with tf.name_scope("train"):
            train_op = tf.train.GradientDescentOptimizer(FLAGS.learning_rate, update_mode=FLAGS.update_mode).minimize(
                cross_entropy, global_step=global_step)
        with tf.name_scope("Accuracy"):
            correct = tf.equal(tf.argmax(y, 1), tf.argmax(y_, 1))
            accuracy = tf.reduce_mean(tf.cast(correct, tf.float32))
        tf.summary.scalar("cost", cross_entropy)
        tf.summary.scalar("accuracy", accuracy)
        summary_op = tf.summary.merge_all()
        init_op = tf.global_variables_initializer()
    return dict(global_step=global_step, x=x, y_=y_, W=[W1, W2, b1, b2], cross_entropy=cross_entropy,
                train_op=train_op, accuracy=accuracy, summary_op=summary_op, init_op=init_op)


def run_graph_worker(server, mnist, logs_path):
    g = build_graph(server.cluster, FLAGS.task_index)
    sv_kw = {}
    if FLAGS.checkpoint_dir:   # the reference passes no logdir, so it can never recover
        sv_kw = dict(logdir=FLAGS.checkpoint_dir, save_model_secs=FLAGS.save_model_secs,
                     save_model_steps=FLAGS.save_model_steps, summary_op=None)
    sv = tf.train.Supervisor(is_chief=server.is_chief, global_step=g["global_step"], init_op=g["init_op"], **sv_kw)
    begin = time.time()
    cost = float("nan")
    steps = 0
    mw = MetricsWriter(FLAGS.metrics_jsonl) if FLAGS.metrics_jsonl else None
    dump = {} if FLAGS.dump_dir else None
    with sv.prepare_or_wait_for_session(server.target) as sess:
        start_gstep = int(sess.run(g["global_step"]))
        if dump is not None:
            dump.update({f"init{k}": np.asarray(sess.run(v)) for k, v in enumerate(g["W"])})
            xs, ys = [], []
        if start_gstep:
            print(f"restored from checkpoint at global step {start_gstep}", flush=True)
        writer = tf.summary.FileWriter(logs_path, graph=tf.get_default_graph())
        batch_count = mnist.train.num_examples // FLAGS.batch_size
        t0 = time.time()
        done = False
        for epoch in range(FLAGS.training_epochs):
            count = 0
            for i in range(batch_count):
                bx, by = mnist.train.next_batch(FLAGS.batch_size)
                if dump is not None:
                    xs.append(np.array(bx, dtype=np.float32))
                    ys.append(np.asarray(by).copy())
                _, cost, summary, step = sess.run([g["train_op"], g["cross_entropy"], g["summary_op"],
                                                   g["global_step"]], feed_dict={g["x"]: bx, g["y_"]: by})
                writer.add_summary(summary, int(step))
                steps += 1
                if steps == 20:
                    t_steady = time.perf_counter()      # per-run cost past the warm-up (dump_dir)
                count += 1
                if mw is not None:
                    mw.write("step", int(step), cost=float(cost))
                if count % FLAGS.frequency == 0 or i + 1 == batch_count:
                    dt = time.time() - t0
                    t0 = time.time()
                    print(step_line(steps, int(sess.run(g["global_step"])), epoch + 1, i + 1, batch_count,
                                    float(cost), dt * 1000.0 / FLAGS.frequency), flush=True)
                    count = 0
                if FLAGS.max_steps and int(step) >= FLAGS.max_steps:   # global steps (resume-aware)
                    done = True
                    break
            if done:
                break
        steady_ms = (time.perf_counter() - t_steady) / (steps - 20) * 1e3 if steps > 20 else None
        acc = float(sess.run(g["accuracy"], feed_dict={g["x"]: mnist.test.images, g["y_"]: mnist.test.labels}))
        if mw is not None:
            mw.write("final", int(sess.run(g["global_step"])), accuracy=acc, cost=float(cost))
            mw.close()
        params = [np.asarray(sess.run(v)) for v in g["W"]]
        gstep = int(sess.run(g["global_step"]))
        writer.close()
        if dump is not None:
            from distributed_tensorflow_example_amd.compat import lowering

            plan = lowering.plan_for(g["train_op"])
            cplan = getattr(plan, "_cplan", None)
            w = server.world
            dump.update({f"final{k}": p for k, p in enumerate(params)})
            dump.update(xs=np.stack(xs), ys=np.stack(ys))
            os.makedirs(FLAGS.dump_dir, exist_ok=True)
            np.savez(os.path.join(FLAGS.dump_dir, f"worker_{FLAGS.task_index}.npz"), **dump)
            with open(os.path.join(FLAGS.dump_dir, f"worker_{FLAGS.task_index}.json"), "w") as f:
                json.dump({"lowered_steps": getattr(plan, "steps", 0) if plan else 0,
                           "native_plan_steps": int(cplan.steps()) if cplan is not None else 0,
                           "native_plan_ipc": bool(cplan.has_ipc()) if cplan is not None else False,
                           "rccl_comm": w is not None and w.comm is not None,
                           "ipc_calls": int(w.ipc.calls()) if w is not None and w.ipc is not None else 0,
                           "ipc_error": w.ipc_error if w is not None else None,
                           "world_size": w.world_size if w is not None else 1,
                           "steps": steps, "session_loop_ms_per_step_after_20": steady_ms}, f)
    sv.stop()
    return acc, float(cost), time.time() - begin, params, gstep


def run_fused_worker(server, mnist):
    """Whole-step MFMA kernel chain (models.mlp) fed from the same dataset."""
    import torch

    from distributed_tensorflow_example_amd.models import mlp

    world = server.world
    tr = mlp.FusedMLPTrainer(batch_size=FLAGS.batch_size, lr=FLAGS.learning_rate, act=FLAGS.activation,
                             world=world)
    if FLAGS.persistent:
        return run_persistent_worker(server, mnist, tr)
    begin = time.time()
    batch_count = mnist.train.num_examples // FLAGS.batch_size
    steps = 0
    loss = float("nan")
    for epoch in range(FLAGS.training_epochs):
        for i in range(batch_count):
            bx, by = mnist.train.next_batch(FLAGS.batch_size)
            xt = torch.from_numpy(bx).to(tr.device)
            yt = torch.from_numpy(by.argmax(1).astype(np.int32)).to(tr.device)
            tr.step_tensors(xt, yt)
            steps += 1
            if steps % FLAGS.frequency == 0 or i + 1 == batch_count:
                m = tr.read_metrics(steps - 1, steps)
                loss = float(m[-1][0])
                print(step_line(steps, tr.global_step, epoch + 1, i + 1, batch_count, loss, 0.0), flush=True)
            if FLAGS.max_steps and steps >= FLAGS.max_steps:
                break
        if FLAGS.max_steps and steps >= FLAGS.max_steps:
            break
    p = mlp.unflatten(tr.get_params().cpu())
    z = mlp.reference_forward(tr.get_params().cpu(), torch.from_numpy(mnist.test.images), FLAGS.activation)
    acc = float((z.argmax(1).numpy() == mnist.test.labels.argmax(1)).mean())
    params = [p[k].numpy() for k in ("weights/Variable", "weights/Variable_1", "biases/Variable",
                                     "biases/Variable_1")]
    server.signal_done()
    return acc, loss, time.time() - begin, params, tr.global_step


def run_persistent_worker(server, mnist, tr):
    """One persistent launch per epoch (csrc/kernels/mlp_persist.hip); the
    per-epoch shuffle of next_batch is re-packed into the pinned epoch and the
    step lines come from the device metrics ring."""
    import torch

    from distributed_tensorflow_example_amd.data.mnist import PinnedEpoch
    from distributed_tensorflow_example_amd.models import mlp

    train = mnist.train
    epoch = PinnedEpoch(train.images_u8, train.labels_u8, FLAGS.batch_size)
    run = mlp.PersistentMLPRunner(tr, epoch, steps_per_launch=epoch.num_batches)
    batch_count = epoch.num_batches
    begin = time.time()
    steps, loss = 0, float("nan")
    for ep in range(FLAGS.training_epochs):
        if ep:
            epoch.shuffle(seed=1000 * FLAGS.task_index + ep)
            run.invalidate()             # the staged chunks came from the previous packing
        n = batch_count if not FLAGS.max_steps else min(batch_count, FLAGS.max_steps - steps)
        if n <= 0:
            break
        g0 = tr.global_step
        run.run(n)
        torch.cuda.synchronize()
        if run.error():
            raise RuntimeError("persistent kernel exchange timed out")
        m = tr.read_metrics(g0, g0 + n)
        dt = run.step_times_ms(g0, g0 + n)   # device per-step stamps (example.py:174-183 AvgTime)
        for i in range(n):
            if (steps + i + 1) % FLAGS.frequency == 0 or i + 1 == batch_count:
                avg = float(dt[max(0, i + 1 - FLAGS.frequency):i + 1].mean())
                print(step_line(steps + i + 1, g0 + i + 1, ep + 1, i + 1, batch_count, float(m[i][0]), avg),
                      flush=True)
        loss = float(m[-1][0])
        steps += n
    z = mlp.reference_forward(tr.get_params().cpu(), torch.from_numpy(mnist.test.images), FLAGS.activation)
    acc = float((z.argmax(1).numpy() == mnist.test.labels.argmax(1)).mean())
    p = mlp.unflatten(tr.get_params().cpu())
    params = [p[k].numpy() for k in ("weights/Variable", "weights/Variable_1", "biases/Variable",
                                     "biases/Variable_1")]
    server.signal_done()
    return acc, loss, time.time() - begin, params, tr.global_step


def main(_argv):
    cluster = cluster_spec()
    server = tf.train.Server(cluster, job_name=FLAGS.job_name, task_index=FLAGS.task_index)
    logs_path = os.path.join(FLAGS.logs_path, f"{FLAGS.job_name}_{FLAGS.task_index}")
    shutil.rmtree(logs_path, ignore_errors=True)
    os.makedirs(logs_path, exist_ok=True)

    if FLAGS.job_name == "ps":
        print(f"ps {FLAGS.task_index} start ...", flush=True)
        server.join()
        print(f"ps {FLAGS.task_index} done", flush=True)
        return 0
    print(f"worker {FLAGS.task_index} start ...", flush=True)
    data_dir = FLAGS.data_dir or f"MNIST_data/{FLAGS.job_name}_{FLAGS.task_index}"
    # the loop below feeds batches unmodified: read-only pixel batches, shipped as uint8 by the lowered step
    mnist = mnist_data.read_data_sets(data_dir, one_hot=True, seed=FLAGS.task_index, train_size=FLAGS.train_size,
                                      pixel_batches=True)
    print(f"MNIST source: {mnist.source} (train {mnist.train.num_examples}, validation "
          f"{mnist.validation.num_examples}, test {mnist.test.num_examples})", flush=True)
    if FLAGS.fused:
        acc, cost, total, params, gstep = run_fused_worker(server, mnist)
    else:
        acc, cost, total, params, gstep = run_graph_worker(server, mnist, logs_path)
    print("Test-Accuracy: %2.2f" % acc)
    print("Total Time: %3.2fs" % total)
    print("Final Cost: %.4f" % cost)
    if FLAGS.result_json:
        with open(FLAGS.result_json, "w") as f:
            json.dump({"accuracy": acc, "cost": cost, "global_step": gstep,
                       "param_sums": [float(np.float64(p).sum()) for p in params],
                       "param_abs": [float(np.abs(np.float64(p)).sum()) for p in params]}, f)
    print("done", flush=True)
    return 0


if __name__ == "__main__":
    tf.app.run(main)
