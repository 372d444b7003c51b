"""tf.logging-compatible logging + the reference's task-prefixed helpers.

Reference: `tf.logging.set_verbosity(INFO)` and `debug/info/error(msg)` that
prefix `[YYYY-mm-dd HH:MM:SS] [job:task]` (lr2.py:13-15,38-48), plus the
example.py console line `Step: .., Global Step: .., Epoch: .., Batch: .. of ..,
Cost: .., AvgTime: ..ms` (example.py:178-183) reproduced by `step_line`.
"""
from __future__ import annotations

import logging as _logging
import sys
import time

DEBUG = _logging.DEBUG
INFO = _logging.INFO
WARN = _logging.WARNING
WARNING = _logging.WARNING
ERROR = _logging.ERROR
FATAL = _logging.CRITICAL

_logger = _logging.getLogger("dtf")
if not _logger.handlers:
    _h = _logging.StreamHandler(sys.stderr)
    _h.setFormatter(_logging.Formatter("%(levelname).1s%(asctime)s %(message)s", "%m%d %H:%M:%S"))
    _logger.addHandler(_h)
    _logger.setLevel(INFO)
    _logger.propagate = False


def set_verbosity(level):
    _logger.setLevel(level)


def get_verbosity():
    return _logger.level


def debug(msg, *a):
    _logger.debug(msg, *a)


def info(msg, *a):
    _logger.info(msg, *a)


def warning(msg, *a):
    _logger.warning(msg, *a)


warn = warning


def error(msg, *a):
    _logger.error(msg, *a)


def fatal(msg, *a):
    _logger.critical(msg, *a)


def log_every_n(level, msg, n, *a):
    c = _counters.get(msg, 0)
    _counters[msg] = c + 1
    if c % n == 0:
        _logger.log(level, msg, *a)


_counters = {}


class TaskLogger:
    """`[time] [job:task] msg` helpers of lr2.py:38-48."""

    def __init__(self, job_name: str, task_index: int):
        self.job, self.task = job_name, int(task_index)

    def _fmt(self, msg):
        tm = time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(time.time()))
        return f" [{tm}] [{self.job}:{self.task}] {msg}"

    def debug(self, msg):
        debug(self._fmt(msg))

    def info(self, msg):
        info(self._fmt(msg))

    def error(self, msg):
        error(self._fmt(msg))


def step_line(step: int, global_step: int, epoch: int, batch: int, batch_count: int, cost: float,
              avg_ms: float) -> str:
    """The example.py:178-183 progress line (same field formats)."""
    return ("Step: %d, " % step + " Global Step: %2d, " % global_step + " Epoch: %2d, " % epoch
            + " Batch: %3d of %3d, " % (batch, batch_count) + " Cost: %.4f, " % cost
            + " AvgTime: %3.2fms" % avg_ms)
