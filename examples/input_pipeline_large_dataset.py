"""Feeder-thread queue demo -- counterpart of input_pipeline_large_dataset.py.

A Python thread enqueues wrap-around chunks of 20 rows of a 100,003 x 4
array (+ one-hot [1,0,0] targets) into FIFOQueue(capacity=50, shapes [4],[3]);
tf.train.batch(15, capacity=40) dequeues under RunOptions(timeout_in_ms=4000)
(input_pipeline_large_dataset.py:9-66).  Unlike the reference (which
`exit(0)`s before its shutdown block, :68-74) the queue is closed with
cancel_pending_enqueues and every thread is joined.
"""
from __future__ import annotations

import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import distributed_tensorflow_example_amd.compat as tf  # noqa: E402

flags = tf.app.flags
flags.DEFINE_integer("batches", 1000, "batches to dequeue")
flags.DEFINE_boolean("verbose", False, "print every batch")
FLAGS = flags.FLAGS


def main(_argv):
    r = np.arange(0.0, 100003.0)
    raw_data = np.dstack((r, r, r, r))[0].astype(np.float32)
    raw_target = np.array([[1, 0, 0]] * 100003, np.float32)
    queue_input_data = tf.placeholder(tf.float32, shape=[20, 4])
    queue_input_target = tf.placeholder(tf.float32, shape=[20, 3])
    queue = tf.FIFOQueue(capacity=50, dtypes=[tf.float32, tf.float32], shapes=[[4], [3]])
    enqueue_op = queue.enqueue_many([queue_input_data, queue_input_target])
    dequeue_op = queue.dequeue()
    data_batch, target_batch = tf.train.batch(dequeue_op, batch_size=15, capacity=40)
    sess = tf.Session()

    def enqueue():
        under, n = 0, len(raw_data)
        try:
            while True:
                upper = under + 20
                if upper <= n:
                    d, t = raw_data[under:upper], raw_target[under:upper]
                    under = upper
                else:
                    rest = upper - n
                    d = np.concatenate((raw_data[under:n], raw_data[:rest]))
                    t = np.concatenate((raw_target[under:n], raw_target[:rest]))
                    under = rest
                sess.run(enqueue_op, feed_dict={queue_input_data: d, queue_input_target: t})
        except tf.errors.CancelledError:
            pass

    feeder = threading.Thread(target=enqueue, daemon=True)
    feeder.start()
    coord = tf.train.Coordinator()
    threads = tf.train.start_queue_runners(coord=coord, sess=sess)
    expect = 0.0
    for i in range(FLAGS.batches):
        d, t = sess.run([data_batch, target_batch], options=tf.RunOptions(timeout_in_ms=4000))
        assert d.shape == (15, 4) and t.shape == (15, 3)
        assert d[0, 0] == expect % 100003          # strict FIFO order through both queues
        expect = (expect + 15) % 100003
        if FLAGS.verbose:
            print(d)
    print(f"dequeued {FLAGS.batches} batches of 15; last row {d[-1]}")
    sess.run(queue.close(cancel_pending_enqueues=True))
    coord.request_stop()
    coord.join(threads, stop_grace_period_secs=5, ignore_live_threads=True)
    feeder.join(5)
    sess.close()
    return 0


if __name__ == "__main__":
    tf.app.run(main)
