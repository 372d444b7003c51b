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
numbers.  One rank keeps up to `max_graphs` signatures (e.g. the compat
Session's lr2 step: a full batch and the epoch's last, shorter one, each at a
few padded id capacities); the least recently used one is dropped beyond that.

A replay returns the graph's static output tensor: it is overwritten by the
next replay (copy it to keep it).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Callable, List, Sequence

import torch


class _Captured:
    __slots__ = ("graph", "static_in", "out")

    def __init__(self, graph, static_in, out):
        self.graph, self.static_in, self.out = graph, static_in, out


class GraphedStep:
    """`strict` (multi-rank steps with collectives): the graph is captured only
    by an explicit `capture(example)` that every rank makes at the same point
    (the capture's warmup iterations run the step's collectives), and a call
    whose input shapes differ from the captured ones raises instead of
    capturing again on one rank alone."""

    def __init__(self, step_fn: Callable, state: Callable[[], Sequence[torch.Tensor]], warmup: int = 2,
                 strict: bool = False, max_graphs: int = 8):
        self.step_fn = step_fn
        self.state = state            # -> the tensors the step mutates (snapshotted around warmup)
        self.warmup = warmup
        self.strict = strict
        self.max_graphs = 1 if strict else max(1, int(max_graphs))
        self._graphs: "OrderedDict[tuple, _Captured]" = OrderedDict()
        self.captures = 0
        self.replays = 0

    @staticmethod
    def _sig(inputs):
        return tuple((tuple(t.shape), t.dtype, t.device) for t in inputs)

    # the most recent capture (tests and callers that hold one signature)
    @property
    def key(self):
        return next(reversed(self._graphs)) if self._graphs else None

    @property
    def graph(self):
        return self._graphs[self.key].graph if self._graphs else None

    @property
    def out(self):
        return self._graphs[self.key].out if self._graphs else None

    def _capture(self, inputs):
        sig = self._sig(inputs)
        self._graphs.pop(sig, None)
        static_in = [t.detach().clone() for t in inputs]
        saved = [t.detach().clone() for t in self.state()]
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self.step_fn(*static_in)
        cur.wait_stream(side)
        from .. import ops
        g = torch.cuda.CUDAGraph()
        ops.bump_capture_epoch()          # no eager-cached sort / bag plan inside the graph
        with torch.cuda.graph(g):
            out = self.step_fn(*static_in)
        ops.bump_capture_epoch()          # nor a captured one in later eager calls
        with torch.no_grad():
            for t, s in zip(self.state(), saved):
                t.copy_(s)
        del saved
        self._graphs[sig] = _Captured(g, static_in, out)
        while len(self._graphs) > self.max_graphs:
            self._graphs.popitem(last=False)
        self.captures += 1

    def capture(self, *inputs):
        """(Re)capture now with `inputs` as the example (state is restored after)."""
        if self.strict:
            self._graphs.clear()
        self._capture(inputs)

    def matches(self, *inputs) -> bool:
        return self._sig(inputs) in self._graphs

    def __call__(self, *inputs):
        sig = self._sig(inputs)
        c = self._graphs.get(sig)
        if c is None:
            if self.strict:
                raise RuntimeError("captured multi-rank step called with other input shapes "
                                   f"({sig} vs {self.key}): pad inputs to the static capacity; a "
                                   "re-capture must be collective (capture() on every rank)")
            self._capture(inputs)
            c = self._graphs[sig]
        else:
            self._graphs.move_to_end(sig)
        with torch.no_grad():
            from .. import ops
            ops.multi_copy_(c.static_in, inputs)      # the inputs' refresh as one kernel
        c.graph.replay()
        self.replays += 1
        return c.out
