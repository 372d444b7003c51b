"""cProfile of the lowered compat Session.run loop (the reference's training
loop shape: sess.run([train_op, cost, global_step], feed_dict=...))."""
import cProfile
import os
import pstats
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import distributed_tensorflow_example_amd.compat as tf  # noqa: E402
from test_lowering_cpu import _graph  # noqa: E402

rng = np.random.default_rng(0)
B = 100
from distributed_tensorflow_example_amd.data.mnist import PixelBatch  # noqa: E402

xs = [PixelBatch.of(u) for u in rng.integers(0, 256, (64, B, 784), dtype=np.uint8)]   # loader-shaped batches
ys = np.eye(10, dtype=np.float32)[rng.integers(0, 10, (64, B))]
g = _graph(tf)
with tf.Session() as sess:
    sess.run(tf.global_variables_initializer())
    fetch = [g["train"], g["ce"], g["gs"]]
    for i in range(50):
        sess.run(fetch, feed_dict={g["x"]: xs[i % 64], g["y_"]: ys[i % 64]})
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for i in range(2000):
        sess.run(fetch, feed_dict={g["x"]: xs[i % 64], g["y_"]: ys[i % 64]})
    torch.cuda.synchronize()
    pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
