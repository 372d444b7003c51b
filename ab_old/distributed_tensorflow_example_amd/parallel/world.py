"""Process-group bootstrap: one process per GPU, RCCL data plane, gloo control plane.

The reference ties every worker to the ps over TF's gRPC runtime
(`tf.train.Server`, example.py:38-40; lr2.py:331).  Here each rank is one
process bound to one MI355X:

* control plane -- `torch.distributed` gloo group (host tensors: barriers,
  object broadcast, timing reductions, RCCL unique-id exchange).  It is also
  the *data* plane on CPU-only hosts (BASELINE config #1, "runs without a GPU").
* data plane    -- on one node, the IPC collectives (csrc/comm/ipc_coll.cpp,
  csrc/kernels/ipc_coll.hip: every rank maps every peer's exported uncached
  buffer and each collective is one kernel that publishes its input, waits
  for the peers' sequence numbers and reads their slots over xGMI) for every
  latency-bound collective and every all-to-all; the native `RcclComm`
  (csrc/comm/rccl_comm.cpp) for large all-reduce / broadcast / all-gather
  payloads when RCCL comes up -- otherwise those run on IPC too, chunked.
  Both issue on the caller's HIP stream and are hipGraph-capturable.
  DTF_DATA_PLANE=ipc | rccl | auto (default) picks; the choice for a call
  depends only on what every rank knows alike (payload size, dtype), so all
  ranks take the same path.

Rendezvous comes from the torchrun env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)
or explicitly (ClusterSpec path in `compat.train.Server`).
"""
from __future__ import annotations

import datetime
import math
import os
import socket
from dataclasses import dataclass, field
from typing import Any, Optional

import torch
import torch.distributed as dist

_WORLD: Optional["World"] = None


@dataclass
class World:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    backend: str = "none"          # "rccl" | "gloo" | "none"
    comm: Any = None               # native RcclComm (GPU data plane); None until ensure_comm() when lazy
    pg_initialized: bool = False
    comm_error: Optional[str] = None   # why the RCCL communicator could not be created (all ranks agree)
    rccl_timeout_s: float = 120.0
    _uid_source: Any = None        # callable(rank) -> RCCL unique id of rank 0 (store- or gloo-based)
    ipc: Any = None                # native IpcColl (the node's RCCL-free data plane); None until ensure_ipc()
    ipc_error: Optional[str] = None    # why the IPC plane is unavailable (all ranks agree)
    data_plane: str = field(default_factory=lambda: os.environ.get("DTF_DATA_PLANE", "auto"))

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    # ------------------------------------------------------------ control plane
    def barrier(self):
        if self.pg_initialized:
            dist.barrier()

    def host_all_reduce(self, value: float, op: str = "sum") -> float:
        if not self.pg_initialized:
            return float(value)
        t = torch.tensor([float(value)], dtype=torch.float64)
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                               "min": dist.ReduceOp.MIN}[op])
        return float(t.item())

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self.pg_initialized:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src)
        return lst[0]

    def all_gather_object(self, obj: Any) -> list:
        if not self.pg_initialized:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj)
        return out

    # --------------------------------------------------------------- data plane
    def ensure_comm(self):
        """Create the RCCL communicator now if this world wants one and has none.

        COLLECTIVE over the world's ranks (every rank must call it at the same
        point: the data-plane methods below do, and so do trainers that issue
        RCCL calls themselves).  Bounded: RCCL's init runs non-blocking and is
        aborted after `rccl_timeout_s`; the ranks agree on the outcome over the
        gloo control plane, so either every rank has a communicator or every rank
        raises RuntimeError (recorded in `comm_error`; later calls re-raise it
        without another attempt).  Returns the communicator, or None for worlds
        without an RCCL data plane (one rank, gloo, CPU).  DTF_FAULT_RCCL_INIT=1
        injects an init failure (tests of the fallback paths)."""
        if self.comm is not None:
            return self.comm
        if self.comm_error is not None:
            raise RuntimeError(self.comm_error)
        fault = os.environ.get("DTF_FAULT_RCCL_INIT", "0") == "1"
        if self.world_size == 1 or not self.pg_initialized or (self.backend != "rccl" and not fault):
            return None
        err = "RCCL init fault injected (DTF_FAULT_RCCL_INIT=1)" if fault else None
        comm = None
        if err is None:
            try:
                from .. import _native

                C = _native.load()
                uid = self._uid_source(self) if self._uid_source is not None else self._gloo_uid(C)
                comm = C.RcclComm(uid, self.world_size, self.rank, float(self.rccl_timeout_s))
            except Exception as e:  # noqa: BLE001
                err = f"RCCL init failed on rank {self.rank}: {e}"
        ok = self.host_all_reduce(0.0 if err is not None else 1.0, "min")
        if ok < 1.0:
            if comm is not None:
                try:
                    comm.abort()
                except Exception:  # noqa: BLE001
                    pass
            self.comm_error = err or "RCCL init failed on a peer rank"
            raise RuntimeError(self.comm_error)
        self.comm = comm
        return comm

    def _gloo_uid(self, C):
        return self.broadcast_object(C.rccl_unique_id() if self.rank == 0 else None, 0)

    def ensure_ipc(self):
        """Create the IPC data plane now if this world can have one: GPU ranks
        that all live on this node (host name + boot id agree) and a data plane
        setting other than "rccl".  COLLECTIVE, like ensure_comm: every rank gets
        an IpcColl or every rank gets None (reason in `ipc_error`).
        DTF_IPC_SLOT_MB (default 64) sizes each of a rank's two payload slots,
        DTF_IPC_TIMEOUT_S (default 60) bounds every wait for a peer."""
        if self.ipc is not None:
            return self.ipc
        if self.ipc_error is not None:
            return None
        if (self.world_size == 1 or not self.pg_initialized or self.device.type != "cuda"
                or self.data_plane == "rccl"):
            return None
        try:
            boot = open("/proc/sys/kernel/random/boot_id").read().strip()
        except OSError:
            boot = ""
        idents = self.all_gather_object((socket.gethostname(), boot))
        if len(set(idents)) != 1:
            self.ipc_error = "ranks span several nodes"
            return None
        from .. import _native

        C = _native.load()
        cap = int(float(os.environ.get("DTF_IPC_SLOT_MB", "64")) * (1 << 20)) // 256 * 256
        try:
            buf = open_peer_buffers(C, C.ipc_coll_buffer_bytes(cap), self)      # collective, agreed
        except RuntimeError as e:
            self.ipc_error = str(e)
            return None
        err = None
        try:
            coll = C.IpcColl(buf, buf.table_ptr(), self.world_size, self.rank, cap,
                             float(os.environ.get("DTF_IPC_TIMEOUT_S", "60")),
                             int(float(os.environ.get("DTF_IPC_TWO_SHOT_KB", "1024")) * 1024),
                             int(os.environ.get("DTF_IPC_GRID", "128")))
        except Exception as e:  # noqa: BLE001
            coll, err = None, f"IpcColl setup failed on rank {self.rank}: {e}"
        if self.host_all_reduce(0.0 if err is not None else 1.0, "min") < 1.0:
            self.ipc_error = err or "IpcColl setup failed on a peer rank"
            return None
        self.ipc = coll
        return coll

    _IPC_DTYPES = (torch.float32, torch.bfloat16, torch.float64, torch.int32, torch.int64)

    def gpu_coll(self, nbytes: int, kind: str = "reduce"):
        """The data plane for one GPU collective of `nbytes` per rank (the same
        on every rank): the IpcColl, the RCCL communicator, or None (gloo).
        kind "a2a" (all-to-all: per-rank sizes differ) always takes IPC when it
        is up.  COLLECTIVE on first use (sets up the planes)."""
        if self.world_size == 1:
            return None
        ipc = self.ensure_ipc() if self.data_plane != "rccl" else None
        if ipc is not None and (self.data_plane == "ipc" or kind == "a2a"
                                or nbytes <= float(os.environ.get("DTF_IPC_AUTO_MB", "8")) * (1 << 20)):
            return ipc
        if self.backend == "rccl" or os.environ.get("DTF_FAULT_RCCL_INIT", "0") == "1":
            if ipc is None:
                self.ensure_comm()            # raises (agreed) if RCCL cannot come up
            else:
                try:
                    self.ensure_comm()
                except RuntimeError:
                    pass                      # large payloads go over IPC, chunked
        if self.comm is not None:
            return self.comm
        return ipc

    @staticmethod
    def _aligned(t: torch.Tensor) -> bool:
        return t.is_contiguous() and t.data_ptr() % 16 == 0

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.world_size == 1:
            return t
        coll = self.gpu_coll(t.numel() * t.element_size()) if t.is_cuda else None
        if coll is not None and coll is self.ipc:
            if t.dtype in self._IPC_DTYPES and self._aligned(t):
                coll.all_reduce(t, op)
            elif t.dtype in self._IPC_DTYPES or t.dtype == torch.float16:
                wide = t.to(torch.float32 if t.dtype == torch.float16 else t.dtype, memory_format=torch.contiguous_format)
                wide = wide.clone() if not self._aligned(wide) else wide
                coll.all_reduce(wide, op)
                t.copy_(wide)
            else:
                raise TypeError(f"all_reduce over the IPC data plane: dtype {t.dtype} not supported")
        elif coll is not None:
            coll.all_reduce(t, op)
        else:
            if op == "avg":
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                t.div_(self.world_size)
            else:
                dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                                       "min": dist.ReduceOp.MIN}[op])
        return t

    @staticmethod
    def _bytes_view(t: torch.Tensor):
        """(contiguous, 16-byte aligned byte tensor padded to whole 4-byte words,
        needs copy-back) for the IPC byte-copy collectives."""
        nb = t.numel() * t.element_size()
        if t.is_contiguous() and t.data_ptr() % 16 == 0 and nb % 4 == 0:
            return t.view(-1).view(torch.uint8) if t.dim() else t.reshape(1).view(torch.uint8), False
        tmp = torch.zeros(-(-nb // 4) * 4, dtype=torch.uint8, device=t.device)
        tmp[:nb].copy_(t.contiguous().reshape(-1).view(torch.uint8))
        return tmp, True

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world_size == 1:
            return t
        coll = self.gpu_coll(t.numel() * t.element_size()) if t.is_cuda else None
        if coll is not None and coll is self.ipc:
            b, back = self._bytes_view(t)
            coll.broadcast(b, src)
            if back:
                nb = t.numel() * t.element_size()
                t.copy_(b[:nb].view(t.dtype).view(t.shape))
        elif coll is not None:
            coll.broadcast(t, src)
        else:
            dist.broadcast(t, src=src)
        return t

    def all_gather(self, src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
        if self.world_size == 1:
            dst.copy_(src.reshape(dst.shape))
            return dst
        nb = src.numel() * src.element_size()
        coll = self.gpu_coll(nb * self.world_size) if src.is_cuda else None
        if coll is not None and coll is self.ipc:
            if nb % 4 == 0 and self._aligned(src) and self._aligned(dst):
                coll.all_gather(src, dst)
            else:
                s8, _ = self._bytes_view(src)
                pb = s8.numel()
                out = torch.empty(pb * self.world_size, dtype=torch.uint8, device=src.device)
                coll.all_gather(s8, out)
                dst.copy_(out.view(self.world_size, pb)[:, :nb].reshape(-1).view(dst.dtype).view(dst.shape))
        elif coll is not None:
            coll.all_gather(src, dst)
        else:
            dist.all_gather_into_tensor(dst, src)
        return dst

    def reduce_scatter(self, src: torch.Tensor, dst: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.world_size == 1:
            dst.copy_(src.reshape(dst.shape))
            return dst
        coll = self.gpu_coll(src.numel() * src.element_size()) if src.is_cuda else None
        if coll is not None and coll is self.ipc:
            full = src.contiguous().clone()
            self.all_reduce(full, op)
            dst.copy_(full.view(self.world_size, -1)[self.rank].view(dst.shape))
        elif coll is not None:
            self.comm.reduce_scatter(src, dst, op)
        else:
            dist.reduce_scatter_tensor(dst, src, op=dist.ReduceOp.SUM)
        return dst

    def all_to_all(self, src: torch.Tensor, send_counts, dst: torch.Tensor, recv_counts) -> torch.Tensor:
        """Uneven all-to-all; counts are in rows (first dimension) per peer."""
        send_counts = [int(c) for c in send_counts]
        recv_counts = [int(c) for c in recv_counts]
        if self.world_size == 1:
            dst[: recv_counts[0]].copy_(src[: send_counts[0]])
            return dst
        inner = math.prod(src.shape[1:]) * src.element_size()     # bytes per row (the same on every rank)
        coll = self.gpu_coll(0, "a2a") if src.is_cuda and inner % 4 == 0 else \
            (self.gpu_coll(1 << 62) if src.is_cuda else None)
        if coll is not None and coll is self.ipc:
            s, d = src, dst
            if not self._aligned(s):
                s = s.contiguous().clone()
            if not self._aligned(d):
                d = torch.empty_like(dst, memory_format=torch.contiguous_format)
            coll.all_to_all(s, send_counts, d, recv_counts)
            if d is not dst:
                dst.copy_(d)
            return dst
        if src.is_cuda and self.comm is not None:
            inner = math.prod(src.shape[1:])   # counts are in rows; RCCL wants elements
            self.comm.all_to_all(src, [c * inner for c in send_counts], dst, [c * inner for c in recv_counts])
        else:
            dist.all_to_all_single(dst, src, output_split_sizes=recv_counts,
                                   input_split_sizes=send_counts)
        return dst

    def shutdown(self):
        global _WORLD
        self.comm = None
        self.ipc = None
        if self.pg_initialized and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass
        self.pg_initialized = False
        if _WORLD is self:
            _WORLD = None


def _cpu_threads(local_world: int):
    """CPU data plane: split the host's cores between co-located ranks (as
    torchrun does with OMP_NUM_THREADS) unless the user chose a count."""
    if "OMP_NUM_THREADS" in os.environ:
        return
    torch.set_num_threads(max(1, min(4, (os.cpu_count() or 1) // max(1, local_world))))


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init(rank: Optional[int] = None, world_size: Optional[int] = None,
         local_rank: Optional[int] = None, master_addr: Optional[str] = None,
         master_port: Optional[int] = None, backend: str = "auto",
         timeout_s: float = 600.0, rccl: Optional[str] = None, rccl_timeout_s: float = 120.0) -> World:
    """Initialise (idempotently) the process world.

    backend: "auto" -> "rccl" when a GPU is visible, else "gloo".
    rccl: "eager" creates the RCCL communicator here; "lazy" (default, or
    $DTF_RCCL_INIT) leaves it to the first `World.ensure_comm()` -- the
    data-plane methods call it only for payloads the IPC plane does not take --
    so a program whose collectives all run on IPC (the compat Session's MLP
    step, the sharded tables' exchanges) never creates an RCCL communicator.
    Either way the init is bounded by `rccl_timeout_s` and failures are agreed
    on by every rank.
    """
    rccl = rccl or os.environ.get("DTF_RCCL_INIT", "lazy")
    global _WORLD
    if _WORLD is not None:
        return _WORLD
    rank = _env_int("RANK", 0) if rank is None else rank
    world_size = _env_int("WORLD_SIZE", 1) if world_size is None else world_size
    local_rank = _env_int("LOCAL_RANK", rank) if local_rank is None else local_rank
    has_gpu = torch.cuda.is_available()
    if backend == "auto":
        backend = "rccl" if has_gpu else "gloo"
    if backend == "rccl" and not has_gpu:
        raise RuntimeError("backend 'rccl' requested but no GPU is visible")

    if has_gpu and backend == "rccl":
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local_rank % max(ndev, 1))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")

    w = World(rank=rank, world_size=world_size, local_rank=local_rank, device=device,
              backend=backend if world_size > 1 else ("rccl" if device.type == "cuda" else "none"),
              rccl_timeout_s=float(rccl_timeout_s))
    if device.type == "cpu":
        _cpu_threads(_env_int("LOCAL_WORLD_SIZE", world_size))
    if world_size > 1:
        if master_addr is not None:
            os.environ["MASTER_ADDR"] = master_addr
        if master_port is not None:
            os.environ["MASTER_PORT"] = str(master_port)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world_size,
                                    timeout=datetime.timedelta(seconds=timeout_s))
        w.pg_initialized = True
        if backend == "rccl" and rccl == "eager":
            w.ensure_comm()
    _WORLD = w
    return w


def init_from_rendezvous(rdv, backend: str = "auto", timeout_s: float = 600.0) -> World:
    """Data-parallel world of the *workers* of a ClusterSpec (ps tasks excluded).

    gloo bootstraps through the native store (NativeStore); the RCCL unique id
    is exchanged through it as well.
    """
    global _WORLD
    if _WORLD is not None:
        return _WORLD
    if not rdv.is_worker:
        raise RuntimeError("only worker tasks join the data-parallel world")
    from .cluster import NativeStore

    rank, world_size = rdv.task_index, rdv.num_workers
    has_gpu = torch.cuda.is_available()
    if backend == "auto":
        backend = "rccl" if has_gpu else "gloo"
    if backend == "rccl":
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(rank % max(ndev, 1))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    w = World(rank=rank, world_size=world_size, local_rank=rank, device=device,
              backend=backend if world_size > 1 else ("rccl" if device.type == "cuda" else "none"))
    if device.type == "cpu":
        _cpu_threads(rdv.cluster.total_tasks())
    if world_size > 1:
        from .cluster import split_address

        host, port = split_address(rdv.cluster.chief_address())
        store = NativeStore(rdv.store, host, port, timeout_s, prefix="dp/")
        dist.init_process_group("gloo", store=store, rank=rank, world_size=world_size,
                                timeout=datetime.timedelta(seconds=timeout_s))
        w.pg_initialized = True
        if backend == "rccl":
            def uid_from_store(world, _n=[0]):
                from .. import _native

                key = f"rccl_uid/{_n[0]}"     # one key per attempt
                _n[0] += 1
                if world.rank == 0:
                    rdv.store.set(key, _native.load().rccl_unique_id())
                return rdv.store.get(key, timeout_s)
            w._uid_source = uid_from_store
            if os.environ.get("DTF_RCCL_INIT", "lazy") == "eager":
                w.ensure_comm()
    _WORLD = w
    return w


def get_world() -> World:
    return _WORLD if _WORLD is not None else init()


def reset():
    global _WORLD
    if _WORLD is not None:
        _WORLD.shutdown()
    _WORLD = None


def open_peer_buffers(C, nbytes: int, world) -> "object":
    """Collective, failure-tolerant setup of `IpcPeerBuffers` (csrc/comm/ipc_peer.cpp)
    on every rank of `world`: every rank joins the handle exchange even if its own
    allocation failed, and all ranks agree on the outcome -- either every rank gets
    its mapped buffers or every rank raises RuntimeError (so a fallback path taken
    afterwards issues the same collectives everywhere)."""
    err, buf, h = None, None, b""
    try:
        buf = C.IpcPeerBuffers(int(nbytes), world.world_size, world.rank)
        h = bytes(buf.handle())
    except Exception as e:  # noqa: BLE001
        err = e
    handles = world.all_gather_object(h)
    if err is None:
        if not all(handles):
            err = RuntimeError("a peer failed to allocate its IPC buffer")
        else:
            try:
                buf.open(list(handles))
            except Exception as e:  # noqa: BLE001
                err = e
    ok = world.host_all_reduce(0.0 if err is not None else 1.0, "min")
    if ok < 1.0:
        if buf is not None:
            try:
                buf.close()
            except Exception:  # noqa: BLE001
                pass
        raise RuntimeError(f"IPC peer buffers unavailable on some rank ({err})")
    return buf

