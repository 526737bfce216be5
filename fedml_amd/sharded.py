"""Multi-GPU server aggregation inside one node.

The reference server is one process (fedml/__init__.py:339-347 forces one
process per silo for the server), so this is new: one process per GPU, the
round's client updates spread over G GPUs, torch.distributed over RCCL/xGMI.

Two partitionings:

client axis (``ClientAxisAggregator``, the north-star mode)
    GPU g holds whole updates of its own clients K_g (they arrive whole per
    client) and computes the fp32 partial Σ_{i∈K_g} fl(p_i·w_i) with the
    GLOBAL weights w_i = n_i / Σ_all n.  One RCCL reduce-scatter(sum) then
    leaves GPU g owning elements [g·N/G, (g+1)·N/G) of the average.  The
    parameter axis is cut into chunks; the reduce-scatter of chunk c runs on a
    communication stream while chunk c+1 is being reduced, so the exchange
    ((G-1)/G · N · 4 B per GPU) hides under the HBM-bound reduction.  The
    addition order across GPUs differs from the single-GPU chain, so results
    carry a stated tolerance (see ``tolerance``).

parameter axis (``ParamAxisAggregator``)
    GPU g holds columns [g·N/G, (g+1)·N/G) of EVERY client and reduces them
    locally in the reference order: zero exchange, bit-exact.  The result is
    sharded exactly like the client-axis result.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import kernels as kn

F32_EPS = 2.0 ** -24


def shard_range(n: int, world: int, rank: int, align: int = 64) -> Tuple[int, int]:
    """Rank's [lo, hi) of an n-element axis, boundaries 64-element aligned."""
    per = (n + world - 1) // world
    per = (per + align - 1) // align * align
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


class ClientAxisAggregator:
    """Client-axis sharded FedAvg over fp32 or bf16 rows.

    rows: this rank's [K_local, L_pad] client rows (any layout; only the first
    ``length`` elements are reduced).  ``aggregate(global_weights_local)``
    returns this rank's shard of the fp32 result (``[shard_len]``) on the
    current stream.
    """

    def __init__(self, rows: torch.Tensor, length: int, group=None, chunks: int = 8, reducer=None):
        """reducer: test hook ``reducer(rows_chunk [K, n], weights, out [n])``
        replacing the HIP kernel, so the partitioning and the collective can be
        exercised with host tensors over gloo (tests/test_sharded_gloo.py)."""
        self.rows = rows
        self.reducer = reducer
        self.on_gpu = rows.is_cuda
        self.dtype = rows.dtype
        self.length = length
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.K = rows.shape[0]
        dev = rows.device
        self.device = dev
        esz = rows.element_size()
        # Chunk c covers [c*chunk_len, (c+1)*chunk_len) of a world*64-aligned
        # padded axis, so every chunk splits into `world` equal, aligned pieces.
        unit = self.world * 64
        padded = (length + unit - 1) // unit * unit
        chunks = max(1, min(chunks, padded // unit))
        chunk_len = (padded // chunks + unit - 1) // unit * unit
        self.chunk_len = chunk_len
        self.bounds: List[Tuple[int, int]] = []
        lo = 0
        while lo < length:
            self.bounds.append((lo, min(length, lo + chunk_len)))
            lo += chunk_len
        self.piece = chunk_len // self.world
        self.partial = torch.zeros(len(self.bounds) * chunk_len, dtype=torch.float32, device=dev)
        self.shard = torch.empty(len(self.bounds) * self.piece, dtype=torch.float32, device=dev)
        if self.on_gpu:
            # per-chunk source pointer tables (row base + chunk offset)
            self.d_ptrs = [kn.upload_i64([rows[i].data_ptr() + lo * esz for i in range(self.K)], dev)
                           for lo, _ in self.bounds]
        elif reducer is None:
            raise ValueError("host rows need a reducer (the HIP kernels read HBM only)")
        # The exchange runs whenever there is more than one rank, or a process
        # group was handed in explicitly (a one-rank RCCL group exercises the
        # comm stream, the async handles and the stream joins on one GPU).
        self.collective = dist.is_initialized() and (self.world > 1 or group is not None)
        # gloo has no device collectives: stage through the host (a rehearsal
        # mode for N ranks sharing one GPU; RCCL is the production backend)
        self.host_staged = self.collective and self.on_gpu and dist.get_backend(group) == "gloo"
        self.comm_stream = torch.cuda.Stream(dev) if self.collective and self.on_gpu and not self.host_staged else None

    def owned_ranges(self) -> List[Tuple[int, int]]:
        """Global element ranges this rank owns, in shard order (one per chunk)."""
        out = []
        for c, (lo, _) in enumerate(self.bounds):
            a = lo + self.rank * self.piece
            out.append((a, a + self.piece))
        return out

    def aggregate(self, weights: Sequence[float], events: Optional[List] = None,
                  comm_events: Optional[List] = None) -> torch.Tensor:
        """weights: the GLOBAL w_i of this rank's K_local clients, in order.
        events[c] / comm_events[c]: (start, end) torch.cuda.Events around
        chunk c's reduction (caller's stream) and its reduce-scatter (the
        comm stream, from the partial being ready to the collective's end)."""
        if not self.on_gpu:
            return self._aggregate_host(weights)
        cur = torch.cuda.current_stream(self.device)
        d_w = kn.weights_for(weights, torch.float32, self.device) if self.K else None
        works = []
        for c, (lo, hi) in enumerate(self.bounds):
            part = self.partial[c * self.chunk_len: c * self.chunk_len + (hi - lo)]
            if events is not None:
                events[c][0].record(cur)
            if self.K == 0:  # a rank without clients this round contributes zeros
                part.zero_()
            elif self.reducer is not None:
                self.reducer(self.rows[:, lo:hi], weights, part)
            else:
                kn.wsum_ptrs(self.dtype, self.d_ptrs[c], d_w, self.K, hi - lo, part, True)
            if events is not None:
                events[c][1].record(cur)
            if self.host_staged:
                src = self.partial[c * self.chunk_len:(c + 1) * self.chunk_len].cpu()
                dst = torch.empty(self.piece, dtype=src.dtype)
                dist.reduce_scatter_tensor(dst, src, op=dist.ReduceOp.SUM, group=self.group)
                self.shard[c * self.piece:(c + 1) * self.piece].copy_(dst)
            elif self.collective:
                # chunk c's exchange overlaps chunk c+1's reduction
                self.comm_stream.wait_stream(cur)
                with torch.cuda.stream(self.comm_stream):
                    if comm_events is not None:
                        comm_events[c][0].record(self.comm_stream)
                    work = dist.reduce_scatter_tensor(
                        self.shard[c * self.piece:(c + 1) * self.piece],
                        self.partial[c * self.chunk_len:(c + 1) * self.chunk_len],
                        op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                    if comm_events is not None:
                        work.wait()  # the comm stream waits for RCCL's own stream: the end event follows it
                        comm_events[c][1].record(self.comm_stream)
                    works.append(work)
            else:
                self.shard[c * self.piece:(c + 1) * self.piece].copy_(
                    self.partial[c * self.chunk_len:(c + 1) * self.chunk_len])
        for w in works:
            w.wait()  # makes the current stream wait for the collective
        if self.comm_stream is not None:
            cur.wait_stream(self.comm_stream)
        return self.shard

    def _aggregate_host(self, weights: Sequence[float]) -> torch.Tensor:
        for c, (lo, hi) in enumerate(self.bounds):
            part = self.partial[c * self.chunk_len: c * self.chunk_len + (hi - lo)]
            if self.K == 0:
                part.zero_()
            else:
                self.reducer(self.rows[:, lo:hi], weights, part)
            src = self.partial[c * self.chunk_len:(c + 1) * self.chunk_len]
            dst = self.shard[c * self.piece:(c + 1) * self.piece]
            if self.collective:
                dist.reduce_scatter_tensor(dst, src, op=dist.ReduceOp.SUM, group=self.group)
            else:
                dst.copy_(src)
        return self.shard

    def shard_in_model_dtype(self) -> torch.Tensor:
        """This rank's shard rounded once (RNE) to the rows' dtype (bf16/f16
        models; fedagg_round_f32 on the GPU, torch's RNE cast for host rows);
        fp32 rows return the fp32 shard itself."""
        if self.dtype in (torch.bfloat16, torch.float16):
            return kn.round_f32(self.shard, self.dtype) if self.on_gpu else self.shard.to(self.dtype)
        return self.shard

    def gather_full(self, shard: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Reassemble the full [length] result on every rank (all-gather of the
        shards; used by tests and when the model must be replicated).  shard:
        a tensor shaped like this rank's shard (default: the fp32 shard; e.g.
        shard_in_model_dtype()'s 16-bit one, gathered widened to fp32, which
        is exact both ways: gloo has no 16-bit types)."""
        src = self.shard if shard is None else shard
        words = src.to(torch.float32) if src.dtype in (torch.bfloat16, torch.float16) else src
        if not self.collective:
            parts = [words]
        elif self.host_staged:
            parts = [torch.empty_like(words, device="cpu") for _ in range(self.world)]
            dist.all_gather(parts, words.cpu(), group=self.group)
            parts = [p.to(words.device) for p in parts]
        else:
            parts = [torch.empty_like(words) for _ in range(self.world)]
            dist.all_gather(parts, words, group=self.group)
        full = torch.empty(len(self.bounds) * self.chunk_len, dtype=words.dtype, device=words.device)
        for c in range(len(self.bounds)):
            for r in range(self.world):
                full[c * self.chunk_len + r * self.piece: c * self.chunk_len + (r + 1) * self.piece] = \
                    parts[r][c * self.piece:(c + 1) * self.piece]
        return full[:self.length].to(src.dtype)

    @staticmethod
    def tolerance(abs_terms_sum: torch.Tensor, k_total: int, world: int) -> torch.Tensor:
        """Per-element bound vs the single-GPU chain: both are sums of the same
        products fl(w_i p_i) in different orders, so
        |Δ| <= 2·(K + log2 G + 1)·2^-24·Σ_i |fl(w_i p_i)|."""
        import math

        return 2.0 * (k_total + math.ceil(math.log2(max(world, 1))) + 1) * F32_EPS * abs_terms_sum


class ParamAxisAggregator:
    """Parameter-axis sharded FedAvg: bit-exact, no collective.

    rows: this rank's [K, L_pad] slice of every client (columns of its shard).
    """

    def __init__(self, rows: torch.Tensor, length: int, reducer=None):
        self.rows = rows
        self.length = length
        self.K = rows.shape[0]
        self.device = rows.device
        self.reducer = reducer
        if rows.is_cuda:
            self.d_ptrs = kn.upload_i64([rows[i].data_ptr() for i in range(self.K)], self.device)
        elif reducer is None:
            raise ValueError("host rows need a reducer (the HIP kernels read HBM only)")
        out_dtype = torch.float32 if rows.dtype == torch.int64 else rows.dtype
        self.out = torch.empty(max(length, 1), dtype=out_dtype, device=self.device)

    def aggregate(self, weights: Sequence[float], events: Optional[List] = None) -> torch.Tensor:
        if self.reducer is not None:
            self.reducer(self.rows[:, :self.length], weights, self.out[:self.length])
            return self.out[:self.length]
        cur = torch.cuda.current_stream(self.device)
        d_w = kn.weights_for(weights, torch.float32, self.device)
        if events is not None:
            events[0][0].record(cur)
        kn.wsum_ptrs(self.rows.dtype, self.d_ptrs, d_w, self.K, self.length, self.out, True)
        if events is not None:
            events[0][1].record(cur)
        return self.out[:self.length]


def buffer_ranges(layout, param_names: Sequence[str]) -> List[Tuple[int, int]]:
    """Element ranges [lo, hi) of the fp32 row that hold BUFFERS (every key
    not among the named parameters: BatchNorm running stats, integer
    counters promoted into the fp32 row), merged where adjacent.  layout: a
    ClientBucket or RowLayout."""
    g = layout.groups[torch.float32]
    params = set(param_names)
    out: List[Tuple[int, int]] = []
    for key, off, n in zip(g.keys, g.offsets, g.numels):
        if n == 0 or key in params:
            continue
        if out and out[-1][1] == off:
            out[-1] = (out[-1][0], off + n)
        else:
            out.append((off, off + n))
    return out


class ShardedFedOpt:
    """Config 5 on G GPUs: FedOpt with the client axis sharded.

    The round's FedAvg is the client-axis mode above (local fp32 partial +
    RCCL reduce-scatter), so rank g ends up owning the average of its
    ``owned_ranges``.  The server optimizer then steps ONLY those elements,
    with the global parameters and the optimizer state (momentum / Adam
    moments / Adagrad sums) sharded the same way: a 1/G slice of the state
    per GPU and no second exchange (gather the parameters with
    ``gather_params`` when the full model is needed, e.g. to broadcast it).

    The step is the fused FedAvg + optimizer kernel with ONE source, the
    reduced shard, at weight 1.0 (fl(x * 1.0) == x), so it is the single-GPU
    server step applied to the multi-GPU average.  As in the reference
    (FedOptAggregator.set_model_global_grads, FedOptAggregator.py:118-130)
    only named parameters are stepped: ``buffers`` lists the element ranges of
    the flat fp32 layout that hold buffers (``buffer_ranges(layout,
    param_names)``), and those take the plain average.  The step runs over
    the whole shard in one launch and the buffer elements are then
    overwritten with the average in one gather/scatter, so a model with
    hundreds of interleaved BatchNorm buffers still costs two launches; the
    optimizer state at buffer positions is never read back.  A LoRA adapter
    set (config 5) has no buffers.

    stepper: test hook ``stepper(param, state: dict, avg)`` replacing the HIP
    step (gloo tests on host rows, tests/test_sharded_gloo.py).
    """

    def __init__(self, rows: torch.Tensor, length: int, global_flat: torch.Tensor, optimizer: str = "sgd",
                 lr: float = 1.0, momentum: float = 0.0, group=None, chunks: int = 8, reducer=None, stepper=None,
                 buffers: Sequence[Tuple[int, int]] = (), weight_decay: Optional[float] = None):
        from .fedopt import (FUSED_OPTIMIZERS, OPTREPO_STATE, _check_momentum, _unsupported, _weight_decay,
                             optrepo_carry)

        self.optimizer = optimizer.lower()
        if self.optimizer not in FUSED_OPTIMIZERS:
            raise _unsupported(optimizer)
        _check_momentum(self.optimizer, momentum)
        self.lr, self.momentum = float(lr), float(momentum) if self.optimizer == "sgd" else 0.0
        self.betas, self.eps = (0.9, 0.999), (1e-10 if self.optimizer == "adagrad" else 1e-8)
        self.alpha = 0.99
        self.weight_decay = _weight_decay(self.optimizer, weight_decay)
        self.agg = ClientAxisAggregator(rows, length, group=group, chunks=chunks, reducer=reducer)
        self.stepper = stepper
        self.length = length
        n = self.agg.shard.numel()
        dev = self.agg.device
        # this rank's slice of the global model, in shard order; padding past
        # `length` stays 0 (its partial sums are 0 as well)
        self.param = torch.zeros(n, dtype=torch.float32, device=dev)
        for c, (a, b) in enumerate(self.agg.owned_ranges()):
            a2, b2 = min(a, length), min(b, length)
            if b2 > a2:
                self.param[c * self.agg.piece: c * self.agg.piece + (b2 - a2)].copy_(global_flat[a2:b2])
        # shard positions of the buffer elements this rank owns
        idx = []
        for c, (a, b) in enumerate(self.agg.owned_ranges()):
            for lo, hi in buffers:
                x, y = max(a, lo), min(b, hi, length)
                if y > x:
                    base = c * self.agg.piece - a
                    idx.append(torch.arange(base + x, base + y, dtype=torch.int64))
        self.buffer_idx = torch.cat(idx).to(dev) if idx else None
        z = lambda: torch.zeros(n, dtype=torch.float32, device=dev)  # noqa: E731
        if self.optimizer == "sgd":
            self.state = {"momentum_buffer": z()} if self.momentum else {}
        elif self.optimizer in ("adam", "adamw"):
            self.state = {"exp_avg": z(), "exp_avg_sq": z()}
        elif self.optimizer == "adagrad":
            self.state = {"sum": z()}
        elif self.optimizer in OPTREPO_STATE:
            self.state = {name: z() for name in OPTREPO_STATE[self.optimizer]}
            if self.optimizer == "rprop":
                self.state["step_size"].fill_(self.lr)
        else:
            self.state = {"square_avg": z()}
        self._carry = optrepo_carry(self.optimizer, self.lr)
        self._names = OPTREPO_STATE.get(self.optimizer, ())
        self.step_count = 0
        if self.agg.on_gpu and stepper is None:
            self._src = kn.upload_i64([self.agg.shard.data_ptr()], dev)  # one source: the reduced shard

    def aggregate(self, weights: Sequence[float], events: Optional[List] = None,
                  comm_events: Optional[List] = None) -> torch.Tensor:
        """One round: weights are the GLOBAL w_i of this rank's clients.
        Returns this rank's updated parameter shard."""
        avg = self.agg.aggregate(weights, events=events, comm_events=comm_events)
        first = self.step_count == 0
        step = self.step_count + 1
        if self.stepper is not None:
            self.stepper(self.param, self.state, avg)
        else:
            n = avg.numel()
            one = kn.HostWeights([1.0])
            if self.optimizer == "sgd":
                kn.wsum_fedopt_sgd(self._src, one, 1, n, self.param, self.state.get("momentum_buffer"), self.lr,
                                   self.momentum, first, True)
            elif self.optimizer == "adam":
                sc = kn.adam_scalars(self.lr, self.betas[0], self.betas[1], self.eps, step)
                kn.wsum_fedopt_adam(self._src, one, 1, n, self.param, self.state["exp_avg"],
                                    self.state["exp_avg_sq"], sc, first, True)
            elif self.optimizer == "adamw":
                sc = kn.adam_scalars(self.lr, self.betas[0], self.betas[1], self.eps, step)
                kn.wsum_fedopt_adamw(self._src, one, 1, n, self.param, self.state["exp_avg"],
                                     self.state["exp_avg_sq"], sc, 1 - self.lr * self.weight_decay, first, True)
            elif self._names:
                osc = kn.optrepo_scalars(self.optimizer, self.lr, step, self._carry)
                kn.wsum_fedopt_optrepo(self.optimizer, self._src, one, 1, n, self.param, self.state[self._names[0]],
                                       self.state[self._names[-1]] if len(self._names) > 1 else None, osc, True)
            elif self.optimizer == "rmsprop":
                kn.wsum_fedopt_rmsprop(self._src, one, 1, n, self.param, self.state["square_avg"], self.lr,
                                       self.alpha, self.eps, True)
            else:
                kn.wsum_fedopt_adagrad(self._src, one, 1, n, self.param, self.state["sum"], self.lr, self.eps, True)
        if self.buffer_idx is not None:  # buffers take the average (FedOptAggregator.py:126-130)
            self.param.index_copy_(0, self.buffer_idx, avg.index_select(0, self.buffer_idx))
        self.step_count = step
        return self.param

    def gather_params(self) -> torch.Tensor:
        """The full [length] global model on every rank (all-gather of the
        parameter shards, reassembled like ClientAxisAggregator.gather_full)."""
        agg = self.agg
        if not agg.collective:
            parts = [self.param]
        elif agg.host_staged:
            parts = [torch.empty_like(self.param, device="cpu") for _ in range(agg.world)]
            dist.all_gather(parts, self.param.cpu(), group=agg.group)
            parts = [p.to(self.param.device) for p in parts]
        else:
            parts = [torch.empty_like(self.param) for _ in range(agg.world)]
            dist.all_gather(parts, self.param, group=agg.group)
        full = torch.empty(len(agg.bounds) * agg.chunk_len, dtype=torch.float32, device=self.param.device)
        for c in range(len(agg.bounds)):
            for r in range(agg.world):
                full[c * agg.chunk_len + r * agg.piece: c * agg.chunk_len + (r + 1) * agg.piece] = \
                    parts[r][c * agg.piece:(c + 1) * agg.piece]
        return full[:self.length]
