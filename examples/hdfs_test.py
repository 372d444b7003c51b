"""Threads counting lines of (fake-)HDFS files through GFile -- hdfs_test.py.

`--files` defaults to three `hdfs://` part files; with DTF_FAKE_HDFS_ROOT set
(tests, no Hadoop here) hdfs:// paths resolve under that directory, else the
`hdfs dfs` CLI backend is used when HADOOP_HDFS_HOME provides it.
"""
from __future__ import annotations

import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_tensorflow_example_amd.compat as tf  # noqa: E402

flags = tf.app.flags
flags.DEFINE_string("files", ",".join(f"hdfs://localhost:9000/user/dtf/lr/data/train/part-{i:05d}"
                                      for i in range(3)), "comma-separated files")
FLAGS = flags.FLAGS


def count_lines(tid, name, out):
    n = 0
    for _ in tf.gfile.GFile(name, mode="r"):
        n += 1
    out[tid] = n
    print("thread: %d, lines: %d, file: %s" % (tid, n, name), flush=True)


def main(_argv):
    names = [f for f in FLAGS.files.split(",") if f]
    out = {}
    threads = [threading.Thread(target=count_lines, args=(i, n, out), daemon=True) for i, n in enumerate(names)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    return 0 if len(out) == len(names) else 1


if __name__ == "__main__":
    tf.app.run(main)
