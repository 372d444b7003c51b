"""hipGraph capture of whole training steps (Session.run / step as
one graph launch instead of dozens of kernel launches from Python).

A step function qualifies when every shape is fixed by the input shapes and
nothing is read back to the host -- e.g. the sparse LR step with the
device-resident routing (parallel/sharded_embedding.py: sort + dedup kernel +
equal-split exchange, no `.tolist()`).  `GraphedStep` captures it once per
input shape signature (warmup iterations on a side stream first, as capture
requires), then each call copies the new inputs into the static buffers and
replays the graph.  The warmup iterations really run the step, so the state
they mutate is snapshotted before and restored after: capturing changes no
numbers.
"""
from __future__ import annotations

from typing import Callable, List, Sequence

import torch


class GraphedStep:
    """`strict` (multi-rank steps with collectives): the graph is captured only
    by an explicit `capture(example)` that every rank makes at the same point
    (the capture's warmup iterations run the step's collectives), and a call
    whose input shapes differ from the captured ones raises instead of
    capturing again on one rank alone."""

    def __init__(self, step_fn: Callable, state: Callable[[], Sequence[torch.Tensor]], warmup: int = 2,
                 strict: bool = False):
        self.step_fn = step_fn
        self.state = state            # -> the tensors the step mutates (snapshotted around warmup)
        self.warmup = warmup
        self.strict = strict
        self.key = None
        self.graph = None
        self.static_in: List[torch.Tensor] = []
        self.out = None
        self.captures = 0
        self.replays = 0

    @staticmethod
    def _sig(inputs):
        return tuple((tuple(t.shape), t.dtype, t.device) for t in inputs)

    def _capture(self, inputs):
        self.graph = None
        self.static_in = [t.detach().clone() for t in inputs]
        saved = [t.detach().clone() for t in self.state()]
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self.step_fn(*self.static_in)
        cur.wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.out = self.step_fn(*self.static_in)
        with torch.no_grad():
            for t, s in zip(self.state(), saved):
                t.copy_(s)
        self.graph = g
        self.key = self._sig(inputs)
        self.captures += 1

    def capture(self, *inputs):
        """(Re)capture now with `inputs` as the example (state is restored after)."""
        self._capture(inputs)

    def matches(self, *inputs) -> bool:
        return self.graph is not None and self._sig(inputs) == self.key

    def __call__(self, *inputs):
        if self.graph is None or self._sig(inputs) != self.key:
            if self.strict:
                raise RuntimeError("captured multi-rank step called with other input shapes "
                                   f"({self._sig(inputs)} vs {self.key}): pad inputs to the static capacity; a "
                                   "re-capture must be collective (capture() on every rank)")
            self._capture(inputs)
        with torch.no_grad():
            for s, t in zip(self.static_in, inputs):
                s.copy_(t, non_blocking=True)
        self.graph.replay()
        self.replays += 1
        return self.out
