"""TF-1.x-shaped front end: `import distributed_tensorflow_example_amd.compat as tf`.

The reference scripts (example.py, lr2.py, model_export.py, the input
pipeline demos) are written against TF 0.12/1.x graph APIs.  This namespace
exposes the subset they use -- with the same names, call signatures and
checkpoint / event-file formats -- on top of the MI355X runtime (fused HIP
kernels, RCCL data plane, native store / queue / IO).  See README for the
behavioural differences (sync instead of async PS, chief-only init).
"""
from __future__ import annotations

import types as _types

from ..utils import flags as _flags
from ..utils import gfile as _gfile
from ..utils import logging as _logging
from . import export as _export
from . import metrics as _metrics
from . import nn
from . import queues as _queues
from . import saver as _saver
from . import summary
from . import train
from .graph import *  # noqa: F401,F403
from .graph import (GLOBAL_VARIABLES, LOCAL_VARIABLES, QUEUE_RUNNERS, SUMMARIES, TRAINABLE_VARIABLES, Graph,
                    Operation, Tensor, Variable, get_default_graph, global_variables_initializer,
                    local_variables_initializer, variables_initializer)
from .partitioned import (PartitionedVariable, fixed_size_partitioner, min_max_variable_partitioner,
                          shard_across_workers, variable_axis_size_partitioner)
from .queues import FIFOQueue, RandomShuffleQueue, decode_jpeg, read_file
from .session import ConfigProto, InteractiveSession, RunMetadata, RunOptions, Session, get_default_session
from .sparse import SparseTensor, SparseTensorValue, sparse_tensor_to_dense

# tf.app ----------------------------------------------------------------------
app = _types.SimpleNamespace(flags=_flags, run=_flags.run)
flags = _flags
logging = _logging
gfile = _types.SimpleNamespace(
    GFile=_gfile.GFile, Open=_gfile.GFile, FastGFile=_gfile.GFile, Exists=_gfile.Exists, Glob=_gfile.Glob,
    ListDirectory=_gfile.ListDirectory, MakeDirs=_gfile.MakeDirs, MkDir=_gfile.MakeDirs,
    Remove=_gfile.Remove, DeleteRecursively=_gfile.DeleteRecursively, Rename=_gfile.Rename,
    Stat=_gfile.Stat, Copy=_gfile.Copy, Walk=_gfile.Walk, IsDirectory=_gfile.IsDirectory)

# tf.errors -------------------------------------------------------------------
errors = _types.SimpleNamespace(OutOfRangeError=_queues.OutOfRangeError,
                                DeadlineExceededError=_queues.DeadlineExceededError,
                                CancelledError=_queues.CancelledError,
                                NotFoundError=FileNotFoundError, InvalidArgumentError=ValueError)

# tf.image / tf.contrib -------------------------------------------------------
image = _types.SimpleNamespace(decode_jpeg=decode_jpeg)
metrics = _types.SimpleNamespace(auc=_metrics.auc, accuracy=_metrics.accuracy)
contrib = _types.SimpleNamespace(
    metrics=_types.SimpleNamespace(streaming_auc=_metrics.streaming_auc,
                                   streaming_accuracy=_metrics.streaming_accuracy),
    session_bundle=_types.SimpleNamespace(exporter=_export, load_session_bundle=_export.load_session_bundle))

# TF 0.x aliases used by the reference (example.py:130-135, lr2.py:408) --------
initialize_all_variables = global_variables_initializer
initialize_local_variables = local_variables_initializer
initialize_variables = variables_initializer
scalar_summary = summary.scalar
histogram_summary = summary.histogram
merge_all_summaries = summary.merge_all
merge_summary = summary.merge
train.SummaryWriter = summary.FileWriter
GraphKeys = _types.SimpleNamespace(GLOBAL_VARIABLES=GLOBAL_VARIABLES, VARIABLES=GLOBAL_VARIABLES,
                                   TRAINABLE_VARIABLES=TRAINABLE_VARIABLES, LOCAL_VARIABLES=LOCAL_VARIABLES,
                                   SUMMARIES=SUMMARIES, QUEUE_RUNNERS=QUEUE_RUNNERS, GLOBAL_STEP="global_step")


def get_collection(key, scope=None):
    return get_default_graph().get_collection(key, scope)


def add_to_collection(key, value):
    get_default_graph().add_to_collection(key, value)
