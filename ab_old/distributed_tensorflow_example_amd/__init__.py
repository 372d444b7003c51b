"""MI355X-native distributed training runtime with the capabilities of
Amano-Ginji/distributed-tensorflow-example (between-graph ps/worker TF example),
re-designed as synchronous data parallelism over RCCL/xGMI with hand-written
CDNA4 HIP kernels.  See README.md / SURVEY.md."""
import torch  # noqa: F401  (load torch's HIP runtime before our extension)

__version__ = "0.1.0"
