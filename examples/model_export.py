"""Linear regression with Adam + model export -- counterpart of model_export.py.

Data x = 0, 0.1, ..., 99.9 and y = x + 20 sin(x / 10) (model_export.py:18-24);
`test/weights` [1,1] ~ N(0,1), `test/bias` [1] = 0; loss = sum((y - xw - b)^2 /
1000) over random batches of 100 drawn with replacement; Adam(0.01) for 500
steps (TF Adam semantics, fused optimizer kernel on GPU); then a Saver-backed
Exporter writes `<work_dir>/<%08d version>/` (session-bundle layout: the
`export.meta` MetaGraphDef carrying the serving signatures + a TF V2 bundle),
and the export is reloaded -- graph rebuilt from the GraphDef, variables
restored -- and served through its signatures as a check.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import distributed_tensorflow_example_amd.compat as tf  # noqa: E402
from distributed_tensorflow_example_amd.compat import export as exporter  # noqa: E402

flags = tf.app.flags
flags.DEFINE_string("work_dir", "./model/", "export base directory")
flags.DEFINE_string("export_version", "0003", "export version")
flags.DEFINE_integer("n_steps", 500, "training steps")
flags.DEFINE_integer("seed", 0, "numpy seed for batch sampling")
FLAGS = flags.FLAGS

N_SAMPLES, LEARNING_RATE, BATCH = 1000, 0.01, 100


def main(_argv):
    rng = np.random.default_rng(FLAGS.seed)
    x_data = np.arange(100, step=0.1).reshape(N_SAMPLES, 1).astype(np.float32)
    y_data = (x_data + 20 * np.sin(x_data / 10)).astype(np.float32)
    x = tf.placeholder(tf.float32, shape=(BATCH, 1), name="x")
    y = tf.placeholder(tf.float32, shape=(BATCH, 1), name="y")
    with tf.variable_scope("test"):
        w = tf.get_variable("weights", (1, 1), initializer=tf.random_normal_initializer(seed=FLAGS.seed))
        b = tf.get_variable("bias", (1,), initializer=tf.constant_initializer(0))
        y_pred = tf.matmul(x, w) + b
        loss = tf.reduce_sum((y - y_pred) ** 2 / N_SAMPLES)
        opt = tf.train.AdamOptimizer(learning_rate=LEARNING_RATE).minimize(loss)
        with tf.Session() as sess:
            sess.run(tf.initialize_all_variables())
            loss_val = None
            for _ in range(FLAGS.n_steps):
                idx = rng.choice(N_SAMPLES, BATCH)
                _, loss_val = sess.run([opt, loss], feed_dict={x: x_data[idx], y: y_data[idx]})
            print(w.eval(sess))
            print(b.eval(sess))
            print(loss_val)
            model_exporter = exporter.Exporter(tf.train.Saver())
            model_exporter.init(sess.graph.as_graph_def(),
                                named_graph_signatures={"inputs": exporter.generic_signature({"x": x}),
                                                        "outputs": exporter.generic_signature({"y": y_pred})})
            path = model_exporter.export(FLAGS.work_dir, tf.constant(FLAGS.export_version), sess)
            wv, bv = sess.run(w), sess.run(b)
    bundle = exporter.load_session_bundle(path)
    probe = np.array([[1.0], [50.0]], np.float32)
    served = bundle.predict(probe).numpy()
    assert np.allclose(served, probe @ wv + bv, atol=1e-5)
    print(f"exported to {path}; signatures {sorted(bundle.signatures)}; served y(50) = {served[1, 0]:.4f}")
    return 0


if __name__ == "__main__":
    tf.app.run(main)
