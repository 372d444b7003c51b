"""Image-file input pipeline demo -- counterpart of input_pipeline.py.

label CSVs (`path,label`) -> first 20 items -> random 5-item test partition
(dynamic_partition) -> slice_input_producer(shuffle=False) -> read_file ->
decode_jpeg(channels=3) -> set_shape([28, 28, 3]) -> batch(5); prints 20
train and 10 test label batches (input_pipeline.py:7-115).  With no dataset
on disk, `--make_synthetic` writes 28x28 RGB JPEGs + CSVs first.  Queue
runners are threads over the native blocking queue; decode is host-side.
"""
from __future__ import annotations

import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import distributed_tensorflow_example_amd.compat as tf  # noqa: E402

flags = tf.app.flags
flags.DEFINE_string("dataset_path", "/tmp/dtf_mnist_jpeg/", "directory with the CSVs and images")
flags.DEFINE_boolean("make_synthetic", True, "create a synthetic JPEG dataset if missing")
flags.DEFINE_integer("train_batches", 20, "train label batches to print")
flags.DEFINE_integer("test_batches", 10, "test label batches to print")
FLAGS = flags.FLAGS

TEST_SET_SIZE, H, W, C, BATCH = 5, 28, 28, 3, 5


def make_synthetic(root, n_train=30, n_test=10, seed=0):
    from PIL import Image

    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "img"), exist_ok=True)
    for name, n in (("train-labels.csv", n_train), ("test-labels.csv", n_test)):
        with open(os.path.join(root, name), "w") as f:
            for i in range(n):
                lab = int(rng.integers(0, 10))
                rel = f"img/{name[:-11]}_{i:04d}.jpg"
                arr = (rng.random((H, W, C)) * 255).astype(np.uint8)
                Image.fromarray(arr).save(os.path.join(root, rel), quality=95)
                f.write(f"{rel},{lab}\n")


def read_label_file(path):
    paths, labels = [], []
    with open(path) as f:
        for line in f:
            p, lab = line.strip().split(",")
            paths.append(p)
            labels.append(int(lab))
    return paths, labels


def main(_argv):
    root = FLAGS.dataset_path
    if FLAGS.make_synthetic and not os.path.exists(os.path.join(root, "train-labels.csv")):
        make_synthetic(root)
    trp, trl = read_label_file(os.path.join(root, "train-labels.csv"))
    tep, tel = read_label_file(os.path.join(root, "test-labels.csv"))
    all_paths = [os.path.join(root, p) for p in trp + tep][:20]
    all_labels = (trl + tel)[:20]
    images = tf.convert_to_tensor(all_paths, dtype=tf.string)
    labels = tf.convert_to_tensor(all_labels, dtype=tf.int32)
    partitions = [0] * len(all_paths)
    partitions[:TEST_SET_SIZE] = [1] * TEST_SET_SIZE
    random.shuffle(partitions)
    train_images, test_images = tf.dynamic_partition(images, partitions, 2)
    train_labels, test_labels = tf.dynamic_partition(labels, partitions, 2)
    train_q = tf.train.slice_input_producer([train_images, train_labels], shuffle=False)
    test_q = tf.train.slice_input_producer([test_images, test_labels], shuffle=False)
    train_image = tf.image.decode_jpeg(tf.read_file(train_q[0]), channels=C)
    test_image = tf.image.decode_jpeg(tf.read_file(test_q[0]), channels=C)
    train_image.set_shape([H, W, C])
    test_image.set_shape([H, W, C])
    train_image_batch, train_label_batch = tf.train.batch([train_image, train_q[1]], batch_size=BATCH)
    test_image_batch, test_label_batch = tf.train.batch([test_image, test_q[1]], batch_size=BATCH)
    print("input pipeline ready")
    with tf.Session() as sess:
        sess.run(tf.initialize_all_variables())
        coord = tf.train.Coordinator()
        threads = tf.train.start_queue_runners(coord=coord, sess=sess)
        print("from the train set:")
        for _ in range(FLAGS.train_batches):
            imgs, labs = sess.run([train_image_batch, train_label_batch])
            assert imgs.shape == (BATCH, H, W, C)
            print(labs)
        print("from the test set:")
        for _ in range(FLAGS.test_batches):
            print(sess.run(test_label_batch))
        coord.request_stop()
        coord.join(threads, stop_grace_period_secs=5, ignore_live_threads=True)
    return 0


if __name__ == "__main__":
    tf.app.run(main)
