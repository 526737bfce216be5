"""Device-resident client-update bucket: the HBM layout of one aggregation round.

The reference keeps every client's update as its own OrderedDict of tensors
and loops over (key, client) pairs (agg_operator.py:36-44); with a GPU server
each tensor is moved to the device as the client arrives
(cross_silo/server/fedml_aggregator.py:58-67 -> ml_engine_adapter.py:234-254).

Here the round's updates live in one row-major [capacity, L] tensor per dtype:
row i is client slot i, every state-dict key sits at a fixed, 16-byte aligned
element offset in the row (rows padded to 64 elements = 256 B; the few
alignment-gap elements are zero and reduce to zero).  ``put`` copies an arriving client's dict straight into its row (the
H2D ingest point), and ``aggregate`` is then one kernel launch per dtype group
over the whole model: for ResNet-50 one fp32 launch over 25,610,152 elements
and one int64 launch over 53.

HBM at config 3 (128 clients x ResNet-50): 128 x 25,610,176 x 4 B = 13.1 GB of
client rows + 102 MB of result, well inside 288 GB; capacity can grow to about
2,700 ResNet-50 clients per GPU.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import weakref
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as nat
from . import kernels as kn
from .layout import RowLayout

_ROW_ALIGN = 64
# host threads for packing a client into pinned staging (the GPU box gives a
# process 16 CPUs; os.cpu_count() reports the whole machine there)
# (8 threads + 3 staging rows: 54 GB/s ingest = 95 % of the measured pinned
# H2D rate, tools/ingest_probe.py; 16 threads contend with the DMA reads)
_PACK_THREADS = int(os.environ.get("FEDAGG_PACK_THREADS", min(8, os.cpu_count() or 1)))
_STAGES = 3
_PIECE = 1 << 22  # columns per evented H2D piece of a put() (16 MiB of fp32)


def _pad(n: int) -> int:
    return (n + _ROW_ALIGN - 1) // _ROW_ALIGN * _ROW_ALIGN


def gather_jobs(jobs: Sequence[dict], threads: int = _PACK_THREADS) -> None:
    """Pack the byte ranges of staging jobs (ClientBucket.put_prepare /
    put_from_table_prepare, of one bucket or of every shard of a
    MultiDeviceBucket) into their pinned rows in ONE native call
    (fedagg_host_gather: one persistent thread pool, no GIL)."""
    parts = [j for j in jobs if j.get("srcs") is not None and len(j["srcs"])]
    if not parts:
        return
    srcs = np.ascontiguousarray(np.concatenate([np.asarray(j["srcs"]).astype(np.uint64, copy=False) for j in parts]))
    dsts = np.ascontiguousarray(np.concatenate([np.asarray(j["dsts"]).astype(np.int64, copy=False) for j in parts]))
    nb = np.ascontiguousarray(np.concatenate([np.asarray(j["nbytes"]).astype(np.int64, copy=False) for j in parts]))
    nat.check(nat.lib().fedagg_host_gather(dsts.ctypes.data, srcs.ctypes.data, nb.ctypes.data, int(nb.size), threads),
              "host_gather")
    for j in parts:
        j["keep"] = None  # converted sources are no longer needed


class ClientBucket:
    """One round's client updates in HBM, laid out for the streaming reduction.

    Args:
        layout: a state dict (OrderedDict of tensors) or a list of
            ``(key, shape, dtype)`` entries, in the model's key order.
        capacity: number of client slots (K).
        device: CUDA device holding the rows.
        low_precision_acc: "reference" (bit-exact with torch's per-op bf16/f16
            rounding) or "fp32" (fp32 accumulate, one final rounding).
        promote_ints: store integer keys in the float32 rows as fl32(v) at
            ingest (default).  The reference computes int64 * w as
            fl32(fl32(v) * fl32(w)) with a float32 result, so this is
            bit-identical and folds e.g. ResNet's 53 counters into the one fp32
            launch.  False keeps exact int64 rows (unweighted integer sums).
    """

    def __init__(self, layout, capacity: int, device=None, low_precision_acc: str = "reference",
                 promote_ints: bool = True):
        if capacity < 1:
            raise ValueError("capacity must be >= 1")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise nat.FedAggNativeError("ClientBucket lives in HBM; give a CUDA device")
        self.capacity = capacity
        self.acc_mode = {"reference": kn.ACC_REFERENCE, "fp32": kn.ACC_FP32}[low_precision_acc]
        self.layout = RowLayout(layout, promote_ints)
        self.entries = self.layout.entries
        self.groups = self.layout.groups
        self.where = self.layout.where
        self.int_keys = self.layout.int_keys
        self.promote_ints = promote_ints
        with torch.cuda.device(self.device):
            for g in self.groups.values():
                g.rows = torch.zeros((capacity, _pad(max(g.length, 1))), dtype=g.dtype, device=self.device)
                g.d_ptrs = kn.upload_i64([g.rows[i].data_ptr() for i in range(capacity)], self.device)
        self.sample_nums: List[Optional[float]] = [None] * capacity
        self._side: Optional[torch.cuda.Stream] = None
        self._copy: Optional[torch.cuda.Stream] = None
        self._staging: Dict[torch.dtype, dict] = {}
        self._result_host: Dict[torch.dtype, torch.Tensor] = {}
        self._pending = False
        # put()'s H2D pieces: per dtype, piece index (column // _PIECE) ->
        # (sequence number, event after the latest copy into it); the copy
        # stream is in order, so that event also covers every earlier copy.
        # _pending_other: an H2D path without pieces is pending
        self._piece_events: Dict[torch.dtype, Dict[int, tuple]] = {}
        self._piece_seq = 0
        self._pending_other = False
        self._d2h: Optional[torch.cuda.Stream] = None
        self._round_outs: Optional[Dict[torch.dtype, torch.Tensor]] = None
        self._plans: Dict[tuple, list] = {}
        self._pool: Optional[Dict[str, torch.Tensor]] = None
        self._pool_thread = None
        # slot -> (client dict, its view dict): dicts whose values a caller
        # bound to this bucket's views (the cross-silo ingest), so a round over
        # them can reduce the rows directly (agg_operator._reduce_resident)
        self._slot_dicts: Dict[int, tuple] = {}
        self._slot_of: Dict[int, int] = {}
        self.entry_keys = [k for k, _, _ in self.entries]
        self._slot_ptrs: Dict[tuple, Dict[torch.dtype, torch.Tensor]] = {}

    # ---- ingest ---------------------------------------------------------------

    def row(self, dtype: torch.dtype, slot: int) -> torch.Tensor:
        g = self.groups[dtype]
        return g.rows[slot, :g.length]

    def view(self, slot: int) -> "OrderedDict[str, torch.Tensor]":
        """Zero-copy views of slot's row, one per key (write a client there)."""
        out = OrderedDict()
        for key, _, _ in self.entries:
            g, j = self.where[key]
            out[key] = g.rows[slot, g.offsets[j]:g.offsets[j] + g.numels[j]].view(g.shapes[j])
        return out

    def put(self, slot: int, state_dict, sample_num: float) -> None:
        """Copy one client's update into its row (FedMLAggregator.
        add_local_trained_result, fedml_aggregator.py:58-67 — the reference
        moves each tensor to the server device there too).

        Device tensors are copied D2D on the current stream.  Host tensors of a
        dtype group are packed into a pinned staging row (one host pass) and
        sent with ONE asynchronous H2D per group on the bucket's copy stream;
        staging is double-buffered, so packing the next client overlaps this
        client's PCIe transfer.  The reduction waits for every pending H2D
        (``sync_ingest``, called by reduce_into)."""
        jobs = self.put_prepare(slot, state_dict, sample_num)
        gather_jobs(jobs)
        self.put_issue(jobs)

    def put_prepare(self, slot: int, state_dict, sample_num: float) -> list:
        """put()'s first half: device tensors are copied D2D now; every dtype
        group with host keys gets a staging job (a pinned row of its ring,
        whose previous H2D has landed, and the byte ranges to gather into
        it).  ``gather_jobs`` packs the jobs of one or several buckets in ONE
        native call and ``put_issue`` sends them: a MultiDeviceBucket packs
        every GPU's keys of an arriving client together and then issues the G
        H2Ds back to back."""
        if not 0 <= slot < self.capacity:
            raise IndexError(f"slot {slot} outside [0, {self.capacity})")
        host: Dict[torch.dtype, List[Tuple[int, int, int, torch.Tensor]]] = {}
        dev_seen: Dict[torch.dtype, int] = {}  # device keys met so far per group: host runs break there
        for key, _, _ in self.entries:
            t = state_dict[key]
            g, j = self.where[key]
            if tuple(t.shape) != g.shapes[j]:
                raise RuntimeError(f"key {key!r}: shape {tuple(t.shape)} != layout {g.shapes[j]}")
            if g.numels[j] == 0:
                continue
            if t.is_cuda:
                src = t.reshape(-1)
                if src.dtype != g.dtype:
                    src = src.to(g.dtype)
                g.rows[slot, g.offsets[j]:g.offsets[j] + g.numels[j]].copy_(src, non_blocking=True)
                dev_seen[g.dtype] = dev_seen.get(g.dtype, 0) + 1
            else:
                host.setdefault(g.dtype, []).append((dev_seen.get(g.dtype, 0), g.offsets[j], g.numels[j], t))
        jobs = [self._stage_prepare(dt, slot, parts) for dt, parts in host.items()]
        self.sample_nums[slot] = sample_num
        return jobs

    def put_issue(self, jobs: list) -> None:
        """put()'s second half: the gathered staging rows' async H2Ds."""
        for job in jobs:
            self._stage_issue(job)

    def put_encoded(self, slot: int, message) -> None:
        """Ingest a FAGG wire message (fedml_amd.wire): its payload already IS
        this bucket's row image, so each dtype group is ONE host->device copy
        straight from the message buffer (asynchronous when the transport
        received it into pinned memory; the runtime stages pageable memory
        itself at ~PCIe rate).  No per-key host work at all.  A pinned message
        buffer must not be rewritten (e.g. by the next receive) before
        sync_ingest() or the reduction has been enqueued and the stream has
        passed it; wait_ingest() blocks the host until then."""
        from . import wire

        if not 0 <= slot < self.capacity:
            raise IndexError(f"slot {slot} outside [0, {self.capacity})")
        sample_num, regions = wire.row_regions(message, self.layout)
        if self._copy is None:
            self._copy = torch.cuda.Stream(self.device)
            self._copy.wait_stream(torch.cuda.current_stream(self.device))
        self._order_after_readers()
        with torch.cuda.stream(self._copy):
            for dt, host in regions:
                if host is not None:
                    self.groups[dt].rows[slot, :host.numel()].copy_(host, non_blocking=True)
        self._pending = True
        self._pending_other = True
        self.sample_nums[slot] = sample_num

    def put_batch(self, tables: Dict[int, bytes], state_dicts: Sequence, sample_nums: Sequence[float]) -> None:
        """Stage ALL capacity slots from host tensors at once: per dtype group
        one native parallel pack of every client's keys into a pinned
        [capacity, padded] image of the rows, then ONE H2D of it on the copy
        stream.  For small rounds, where per-client calls cost more than the
        bytes (config 2: 32 clients x 10 keys).

        tables: {FEDAGG_DT code: int64 host pointers [T_code][capacity]} of the
        keys of that dtype in layout order (walker.walk_host), taken from
        state_dicts; integer keys promoted into the fp32 rows are converted
        from state_dicts per client instead."""
        code_dt = {nat.DT_F32: torch.float32, nat.DT_BF16: torch.bfloat16, nat.DT_F16: torch.float16,
                   nat.DT_F64: torch.float64, nat.DT_I64: torch.int64}
        K = self.capacity
        if len(sample_nums) != K:
            raise ValueError("put_batch stages every slot")
        if self._copy is None:
            self._copy = torch.cuda.Stream(self.device)
            self._copy.wait_stream(torch.cuda.current_stream(self.device))
        ptrs_by_dt = {code_dt[c]: np.frombuffer(t, dtype=np.int64) for c, t in tables.items()}
        for dt, g in self.groups.items():
            if g.length == 0:
                continue
            st = self._staging.get(("batch", dt))
            if st is None:
                st = self._staging[("batch", dt)] = [torch.zeros(g.rows.shape, dtype=dt).pin_memory(), None]
            if st[1] is not None:
                st[1].synchronize()  # the previous round's H2D from this image has landed
            stage = st[0]
            esz = stage.element_size()
            row_bytes = stage.shape[1] * esz
            native = [j for j, k in enumerate(g.keys) if k not in self.int_keys]
            if native:
                ptr = ptrs_by_dt[dt]
                if ptr.size != len(native) * K:
                    raise ValueError("put_batch: pointer table does not match the layout")
                offs = (np.arange(K, dtype=np.int64)[None, :] * row_bytes
                        + np.asarray([g.offsets[j] for j in native], dtype=np.int64)[:, None] * esz).ravel()
                nb = np.repeat(np.asarray([g.numels[j] for j in native], dtype=np.int64) * esz, K)
                live = nb > 0
                srcs, offs, nb = np.ascontiguousarray(ptr[live]), np.ascontiguousarray(offs[live]), nb[live]
                n = int(srcs.size)
                if n:
                    nat.check(nat.lib().fedagg_host_pack(stage.data_ptr(), srcs.ctypes.data, offs.ctypes.data,
                                                         nb.ctypes.data, n, _PACK_THREADS), "host_pack")
            ints = [j for j, k in enumerate(g.keys) if k in self.int_keys]
            for j in ints:  # fl32(v), as the reference's int64 * float promotion sees it
                lo, hi = g.offsets[j], g.offsets[j] + g.numels[j]
                for i in range(K):
                    stage[i, lo:hi].copy_(state_dicts[i][g.keys[j]].reshape(-1))
            self._order_after_readers()
            with torch.cuda.stream(self._copy):
                g.rows.copy_(stage, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._copy)
            st[1] = ev
            self._pending = True
            self._pending_other = True
        for i, n in enumerate(sample_nums):
            self.sample_nums[i] = n

    def put_from_table(self, slot: int, tables: Dict[int, "np.ndarray"], state_dict, sample_num: float,
                       col: Optional[int] = None) -> None:
        """put() for one client of a walked host round: the walker's pointer
        tables (``{code: int64 [T_code, capacity]}``) give every key's host
        pointer, so each dtype group is ONE native pack into a pinned staging
        row of the ring plus ONE async H2D, with no per-key Python work apart
        from integer keys promoted into the fp32 rows (converted from
        state_dict).  col: the tables' column holding this client (default:
        slot; 0 for a table walked from this one dict)."""
        jobs = self.put_from_table_prepare(slot, tables, state_dict, sample_num, col)
        gather_jobs(jobs)
        self.put_issue(jobs)

    def put_from_table_prepare(self, slot: int, tables: Dict[int, "np.ndarray"], state_dict,
                               sample_num: float, col: Optional[int] = None) -> list:
        """put_from_table()'s first half (as put_prepare): per dtype group a
        staging job whose sources are the walker table's pointers of this
        slot; promoted integer keys are converted into the staging row here."""
        code_dt = {nat.DT_F32: torch.float32, nat.DT_BF16: torch.bfloat16, nat.DT_F16: torch.float16,
                   nat.DT_F64: torch.float64, nat.DT_I64: torch.int64}
        if self._copy is None:
            self._copy = torch.cuda.Stream(self.device)
            self._copy.wait_stream(torch.cuda.current_stream(self.device))
        plans = self._table_plans()
        by_dt = {code_dt[c]: t for c, t in tables.items()}
        jobs = []
        for dt, g in self.groups.items():
            if g.length == 0:
                continue
            native, offs, nb, ints = plans[dt]
            b = self._ring_row(dt, g)
            stage = b[0]
            job = {"dt": dt, "slot": slot, "buf": b, "whole": True, "keep": None}
            if native.size:
                job["srcs"] = np.ascontiguousarray(by_dt[dt][native, slot if col is None else col])
                job["dsts"] = offs + stage.data_ptr()
                job["nbytes"] = nb
            for key, lo, n in ints:
                stage[lo:lo + n].copy_(state_dict[key].reshape(-1))
            jobs.append(job)
        self.sample_nums[slot] = sample_num
        return jobs

    def _ring_row(self, dt: torch.dtype, g) -> list:
        """The next pinned staging row of dtype group g's ring, once its
        previous H2D has landed: [row, event of its last H2D]."""
        st = self._staging.get(dt)
        if st is None:  # per dtype group: _STAGES pinned rows used round-robin
            st = self._staging[dt] = {"bufs": [[torch.empty(g.length, dtype=dt).pin_memory(), None]
                                               for _ in range(_STAGES)], "next": 0}
        b = st["bufs"][st["next"]]
        st["next"] = (st["next"] + 1) % _STAGES
        if b[1] is not None:
            b[1].synchronize()  # this staging row's previous H2D has landed
        return b

    def _table_plans(self):
        """Per dtype group: the rows of the walker's table that feed it (keys of
        that dtype with data), their byte offsets and sizes in the row, and the
        promoted integer keys (key, element offset, count)."""
        if getattr(self, "_tplans", None) is None:
            plans = {}
            for dt, g in self.groups.items():
                esz = torch.empty((), dtype=dt).element_size()
                native, offs, nb, ints = [], [], [], []
                r = 0
                for key, off, n in zip(g.keys, g.offsets, g.numels):
                    if key in self.int_keys:
                        if n:
                            ints.append((key, off, n))
                        continue
                    if n:
                        native.append(r)
                        offs.append(off * esz)
                        nb.append(n * esz)
                    r += 1
                plans[dt] = (np.asarray(native, dtype=np.int64), np.asarray(offs, dtype=np.int64),
                             np.asarray(nb, dtype=np.int64), ints)
            self._tplans = plans
        return self._tplans

    def _stage_prepare(self, dt: torch.dtype, slot: int, parts) -> dict:
        g = self.groups[dt]
        if self._copy is None:
            self._copy = torch.cuda.Stream(self.device)
            self._copy.wait_stream(torch.cuda.current_stream(self.device))  # rows were zero-filled there
        b = self._ring_row(dt, g)
        stage = b[0]
        # parts: (run, element offset, count, tensor) in layout order; a run
        # is a stretch of host keys with no device key between them, and each
        # run is ONE H2D of its span: never over a device key's range, which
        # put() already copied D2D (the staging there holds stale bytes)
        runs: Dict[int, List[int]] = {}
        for run, off, n, _ in parts:
            r = runs.setdefault(run, [off, off + n])
            r[0], r[1] = min(r[0], off), max(r[1], off + n)
        esz = stage.element_size()
        base = stage.data_ptr()
        keep = []
        srcs, dsts, nbytes = [], [], []
        for _, off, n, t in parts:
            src = t.reshape(-1)
            if src.dtype != dt or not src.is_contiguous():
                src = src.to(dt).contiguous()
                keep.append(src)
            srcs.append(src.data_ptr())
            dsts.append(base + off * esz)
            nbytes.append(n * esz)
        return {"dt": dt, "slot": slot, "buf": b, "whole": False, "runs": sorted(runs.values()), "keep": keep,
                "srcs": np.asarray(srcs, dtype=np.uint64), "dsts": np.asarray(dsts, dtype=np.int64),
                "nbytes": np.asarray(nbytes, dtype=np.int64)}

    def _stage_issue(self, job: dict) -> None:
        """The H2D of a gathered staging job on the copy stream: a put() job
        in pieces of _PIECE columns, each with an event (the pipelined round
        end starts reducing a column range as soon as the last client's bytes
        for it have landed); a walked-table job as one copy of the row."""
        dt, slot, b = job["dt"], job["slot"], job["buf"]
        g = self.groups[dt]
        stage = b[0]
        self._order_after_readers()
        with torch.cuda.stream(self._copy):
            if job["whole"]:
                g.rows[slot, :g.length].copy_(stage[:g.length], non_blocking=True)
            else:
                last = self._piece_events.setdefault(dt, {})
                for a, e in job["runs"]:
                    while a < e:
                        p = a // _PIECE
                        z = min(e, (p + 1) * _PIECE)
                        g.rows[slot, a:z].copy_(stage[a:z], non_blocking=True)
                        pev = torch.cuda.Event()
                        pev.record(self._copy)
                        self._piece_seq += 1
                        last[p] = (self._piece_seq, pev)
                        a = z
            ev = torch.cuda.Event()
            ev.record(self._copy)
        b[1] = ev
        self._pending = True
        if job["whole"]:
            self._pending_other = True

    def _order_after_readers(self) -> None:
        """An H2D into the rows must not overtake work already enqueued on the
        caller's stream that reads them (the previous round's reduction when
        the next update arrives before it finished): the copy stream waits for
        the current stream first.  A GPU-side wait, no host synchronisation."""
        self._copy.wait_stream(torch.cuda.current_stream(self.device))

    def wait_ingest(self) -> None:
        """Block the host until every H2D issued by the put paths has landed
        (the caller may then reuse its pinned receive buffers)."""
        if self._copy is not None:
            self._copy.synchronize()

    def sync_ingest(self) -> None:
        """Make the current stream wait for every H2D issued by put()."""
        if self._pending and self._copy is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._copy)
        self._ingest_consumed()

    def _ingest_consumed(self) -> None:
        self._pending = False
        self._pending_other = False
        self._piece_events = {}

    # ---- reduction ------------------------------------------------------------

    def weights(self, sample_nums: Sequence[float]) -> List[float]:
        """w_i = n_i / Σn as Python floats (agg_operator.py:24-28, :39)."""
        training_num = 0
        for n in sample_nums:
            training_num += n
        return [n / training_num for n in sample_nums]

    def new_outputs(self) -> Dict[torch.dtype, torch.Tensor]:
        with torch.cuda.device(self.device):
            return {dt: torch.empty(_pad(max(g.length, 1)), dtype=g.out_dtype, device=self.device)
                    for dt, g in self.groups.items()}

    def bind_slot(self, slot: int, state_dict, view) -> None:
        """Record that ``state_dict``'s values are now ``view``'s (this slot's
        views): a later round over such dicts may reduce the rows in place."""
        old = self._slot_dicts.get(slot)
        if old is not None:
            self._slot_of.pop(id(old[0]), None)
        self._slot_dicts[slot] = (state_dict, view)
        self._slot_of[id(state_dict)] = slot

    def reduce_slots(self, slots: Sequence[int], weights: Sequence[float]) -> "OrderedDict[str, torch.Tensor]":
        """FedAvg of the given slots' rows, in that order: per-key device
        tensors (views of one fresh flat buffer per dtype group)."""
        with torch.cuda.device(self.device):
            outs = self.new_outputs()
            self.reduce_into(outs, weights, len(slots), slots=slots)
            return self.unflatten(outs)

    def slot_ptrs(self, slots: Sequence[int]) -> Dict[torch.dtype, torch.Tensor]:
        """Per dtype group, the device table of the given slots' row pointers
        (rows in that order; cached per slot list)."""
        key = tuple(slots)
        t = self._slot_ptrs.get(key)
        if t is None:
            if len(self._slot_ptrs) >= 8:
                self._slot_ptrs.pop(next(iter(self._slot_ptrs)))
            with torch.cuda.device(self.device):
                t = {dt: kn.upload_i64([g.rows[s].data_ptr() for s in slots], self.device)
                     for dt, g in self.groups.items()}
            self._slot_ptrs[key] = t
        return t

    def reduce_into(self, outs: Dict[torch.dtype, torch.Tensor], weights: Sequence[float],
                    num_clients: Optional[int] = None, events: Optional[Dict[torch.dtype, Sequence]] = None,
                    slots: Optional[Sequence[int]] = None) -> None:
        """Launch the weighted sum of rows [0, K) into the flat outputs: one
        kernel per dtype group, on the current stream, no host sync.  events
        maps a dtype to (start, end) torch.cuda.Events recorded around that
        group's launch (the benchmark's per-kernel timing).  slots: the rows
        to reduce, in this order (default 0 .. K-1)."""
        K = num_clients if num_clients is not None else (len(slots) if slots is not None else self.capacity)
        if slots is not None and (len(slots) != K or any(not 0 <= s < self.capacity for s in slots)):
            raise ValueError("slots: one valid slot per client")
        if slots is not None and list(slots) == list(range(K)):
            slots = None
        if not 1 <= K <= self.capacity and slots is None:
            raise ValueError(f"num_clients {K} outside [1, {self.capacity}]")
        if len(weights) != K:
            raise ValueError("one weight per client")
        tables = self.slot_ptrs(slots) if slots is not None else None
        with torch.cuda.device(self.device):
            self.sync_ingest()
            cur = torch.cuda.current_stream(self.device)
            # K <= 256: weights ride in the kernel arguments (no H2D per round)
            w32 = kn.weights_for(weights, torch.float32, self.device)
            w64 = kn.weights_for(weights, torch.float64, self.device) if torch.float64 in self.groups else None
            # The dominant group runs on the caller's stream; the small ones
            # (e.g. ResNet's 53 int64 counters) on a side stream beside it, so
            # their latency-bound launches stay off the critical path.
            dom = self.dominant_dtype()
            minor = [dt for dt, g in self.groups.items() if dt != dom and g.length]
            if minor:
                if self._side is None:
                    self._side = torch.cuda.Stream(self.device)
                self._side.wait_stream(cur)
            # streams passed explicitly (no stream context per launch: ~6 us
            # each, which a one-process round over G GPUs pays G times before
            # the last device starts)
            for dt, g in self.groups.items():
                if g.length == 0:
                    continue
                ev = events.get(dt) if events else None
                s = cur if dt == dom else self._side
                if ev is not None:
                    ev[0].record(s)
                if tables is not None:
                    # a cached table may be read on another stream than the one
                    # it was uploaded on: evicted later, its block must wait for
                    # this launch too
                    tables[dt].record_stream(s)
                kn.wsum_ptrs(dt, g.d_ptrs if tables is None else tables[dt], w64 if dt == torch.float64 else w32,
                             K, g.length, outs[dt], True, self.acc_mode, s.cuda_stream)
                if ev is not None:
                    ev[1].record(s)
            if minor:
                cur.wait_stream(self._side)

    def dominant_dtype(self) -> torch.dtype:
        """The group with the most bytes per client (the roofline kernel)."""
        return max(self.groups.items(), key=lambda kv: kv[1].length * kv[1].rows.element_size())[0]

    def unflatten(self, outs: Dict[torch.dtype, torch.Tensor]) -> "OrderedDict[str, torch.Tensor]":
        """Per-key views of the flat outputs, in the layout's key order."""
        res = OrderedDict()
        for key, _, _ in self.entries:
            g, j = self.where[key]
            res[key] = outs[g.dtype][g.offsets[j]:g.offsets[j] + g.numels[j]].view(g.shapes[j])
        return res

    def aggregate(self, sample_nums: Optional[Sequence[float]] = None, num_clients: Optional[int] = None
                  ) -> "OrderedDict[str, torch.Tensor]":
        """FedAvg over the first K slots; returns device tensors (views of one
        flat buffer per dtype; ``.clone()`` a key to detach it)."""
        K = num_clients if num_clients is not None else self.capacity
        ns = list(sample_nums) if sample_nums is not None else self.sample_nums[:K]
        if any(n is None for n in ns):
            raise ValueError("sample count missing for some slot")
        outs = self.new_outputs()
        self.reduce_into(outs, self.weights(ns), K)
        return self.unflatten(outs)

    # ---- accounting -----------------------------------------------------------

    def algorithmic_bytes(self, num_clients: Optional[int] = None) -> int:
        """Bytes one aggregation must move at minimum: every client element read
        once, every result element written once."""
        K = num_clients if num_clients is not None else self.capacity
        tot = 0
        for g in self.groups.values():
            tot += K * g.length * g.rows.element_size() + g.length * torch.empty((), dtype=g.out_dtype).element_size()
        return tot

    def num_elements(self) -> int:
        """State-dict elements per client (excluding alignment gaps)."""
        return sum(sum(g.numels) for g in self.groups.values())

    # ---- results to the host ----------------------------------------------------

    def to_host(self, outs: Dict[torch.dtype, torch.Tensor], into: Optional[Dict[str, torch.Tensor]] = None
                ) -> "OrderedDict[str, torch.Tensor]":
        """The averaged model as independent host tensors: one D2H per dtype
        group into pinned memory, then a parallel native scatter into one
        tensor per key (each key owns its storage, as the reference's results
        do, so pickling for broadcast sends each key once).

        into: existing contiguous host tensors of the result dtypes (e.g. the
        server model's state_dict, which the reference fills with
        load_state_dict right after aggregating) to write instead of
        allocating: fresh host pages cost a first-touch fault each."""
        res = OrderedDict()
        with torch.cuda.device(self.device):
            for dt, g in self.groups.items():
                h = self._result_host.get(dt)
                if h is None:
                    h = self._result_host[dt] = torch.empty(max(g.length, 1), dtype=g.out_dtype).pin_memory()
                h[:g.length].copy_(outs[dt][:g.length])  # synchronous: needed on the host now
        per_key = {}
        for dt, g in self.groups.items():
            h = self._result_host[dt]
            esz = h.element_size()
            ts, offs, nbytes = [], [], []
            for key, off, n, shape in zip(g.keys, g.offsets, g.numels, g.shapes):
                t = into.get(key) if into is not None else None
                if t is None or t.dtype != g.out_dtype or not t.is_contiguous() or t.is_cuda \
                        or tuple(t.shape) != tuple(shape):
                    t = torch.empty(shape, dtype=g.out_dtype)
                per_key[key] = t
                if n:
                    ts.append(t.data_ptr())
                    offs.append(off * esz)
                    nbytes.append(n * esz)
            n = len(ts)
            if n:
                nat.check(nat.lib().fedagg_host_unpack(h.data_ptr(), (ctypes.c_void_p * n)(*ts),
                                                       (ctypes.c_int64 * n)(*offs), (ctypes.c_int64 * n)(*nbytes),
                                                       n, _PACK_THREADS), "host_unpack")
        for key, _, _ in self.entries:
            res[key] = per_key[key]
        return res

    # ---- round end, pipelined ------------------------------------------------------

    def reduce_to_host(self, weights: Sequence[float], num_clients: Optional[int] = None,
                       into: Optional[Dict[str, torch.Tensor]] = None, chunks: int = 8,
                       timings: Optional[dict] = None) -> "OrderedDict[str, torch.Tensor]":
        """reduce_into + to_host with the three stages overlapped: the dominant
        group is reduced in ``chunks`` column ranges on the current stream;
        each range's D2H into pinned memory runs on a copy stream as soon as
        its kernel ends, and the host scatters a range into the per-key
        tensors as soon as its D2H lands, while the GPU reduces and copies the
        next ones.  Serially the three are ~2 ms (HBM) + ~2 ms (PCIe) + the
        scatter at config 3.  The per-key host tensors come from a pool
        allocated and touched by a background thread after the previous call
        (a fresh tensor pays a page fault per 4 KiB on first write, the bulk
        of the scatter); ``into`` as in to_host.  Same results as
        reduce_into + to_host (the chunked launches are the same per-element
        chains)."""
        return self.finish_to_host(self.launch_to_host(weights, num_clients, into, chunks, timings))

    def launch_to_host(self, weights: Sequence[float], num_clients: Optional[int] = None,
                       into: Optional[Dict[str, torch.Tensor]] = None, chunks: int = 8,
                       timings: Optional[dict] = None) -> tuple:
        """The GPU half of reduce_to_host: every reduction and D2H enqueued,
        nothing waited for.  finish_to_host(state) then scatters into the
        per-key host tensors.  A multi-device bucket launches every device's
        half before finishing any (fedml_amd.multidev)."""
        K = num_clients if num_clients is not None else self.capacity
        if not 1 <= K <= self.capacity:
            raise ValueError(f"num_clients {K} outside [1, {self.capacity}]")
        if len(weights) != K:
            raise ValueError("one weight per client")
        pooled = into is None
        if pooled:
            into = self._take_result_pool()
        per_key = self._host_results(into)
        dom = self.dominant_dtype()
        g = self.groups[dom]
        t = {} if timings is None else timings
        with torch.cuda.device(self.device):
            cur = torch.cuda.current_stream(self.device)
            # only put()'s pieces pending: each range waits for the pieces it
            # covers (the last client's H2D overlaps the first ranges' reduction)
            fine = self._pending and not self._pending_other and self._copy is not None
            if not fine:
                self.sync_ingest()
            pieces = self._piece_events.get(dom, {}) if fine else {}
            if self._d2h is None:
                self._d2h = torch.cuda.Stream(self.device)
            w32 = kn.weights_for(weights, torch.float32, self.device)
            w64 = kn.weights_for(weights, torch.float64, self.device) if torch.float64 in self.groups else None
            outs = self._round_outputs()
            plan = self._chunk_plan(dom, chunks)
            done = []
            for lo, hi, d_ptrs, _ in plan:
                if fine:
                    cover = [pieces[p] for p in range(lo // _PIECE, (hi - 1) // _PIECE + 1) if p in pieces]
                    if cover:  # the copy stream is in order: the latest of them covers the others
                        cur.wait_event(max(cover, key=lambda se: se[0])[1])
                if hi > lo:  # (a round of empty keys only: nothing to launch, empty results)
                    kn.wsum_ptrs(dom, d_ptrs, w64 if dom == torch.float64 else w32, K, hi - lo, outs[dom][lo:hi],
                                 True, self.acc_mode)
                ev = torch.cuda.Event()
                ev.record(cur)
                self._d2h.wait_event(ev)
                h = self._pinned_result(dom)
                with torch.cuda.stream(self._d2h):
                    h[lo:hi].copy_(outs[dom][lo:hi], non_blocking=True)
                    fin = torch.cuda.Event()
                    fin.record(self._d2h)
                done.append(fin)
            if fine:  # everything after this (the small groups, later readers) sees every H2D
                cur.wait_stream(self._copy)
                self._ingest_consumed()
            # the small groups behind the dominant one (e.g. ResNet's counters
            # are promoted into it; bf16 models' fp32 keys are not)
            minor = [dt for dt, gg in self.groups.items() if dt != dom and gg.length]
            for dt in minor:
                gg = self.groups[dt]
                kn.wsum_ptrs(dt, gg.d_ptrs, w64 if dt == torch.float64 else w32, K, gg.length, outs[dt], True,
                             self.acc_mode)
            t["launched"] = True
        return pooled, per_key, dom, plan, done, minor, outs

    def finish_to_host(self, state: tuple) -> "OrderedDict[str, torch.Tensor]":
        """The host half of reduce_to_host (see launch_to_host)."""
        pooled, per_key, dom, plan, done, minor, outs = state
        g = self.groups[dom]
        with torch.cuda.device(self.device):
            dst = np.array([per_key[k].data_ptr() for k in g.keys], dtype=np.int64)
            src = self._pinned_result(dom).data_ptr()
            for (lo, hi, _, (idx, src_off, dst_off, nbytes)), fin in zip(plan, done):
                fin.synchronize()
                n = len(idx)
                if n:
                    dsts = np.ascontiguousarray(dst[idx] + dst_off)
                    nat.check(nat.lib().fedagg_host_unpack(src, dsts.ctypes.data, src_off.ctypes.data,
                                                           nbytes.ctypes.data, n, _PACK_THREADS), "host_unpack")
            for dt in minor:
                gg = self.groups[dt]
                h = self._pinned_result(dt)
                h[:gg.length].copy_(outs[dt][:gg.length])  # synchronous; small
                self._unpack_group(gg, h, per_key)
        if pooled:
            self._refill_result_pool()
        res = OrderedDict()
        for key, _, _ in self.entries:
            res[key] = per_key[key]
        return res

    def _round_outputs(self) -> Dict[torch.dtype, torch.Tensor]:
        """Device outputs reused across reduce_to_host calls (results leave as
        host tensors, so nothing holds them)."""
        if self._round_outs is None:
            self._round_outs = self.new_outputs()
        return self._round_outs

    def _pinned_result(self, dt: torch.dtype) -> torch.Tensor:
        h = self._result_host.get(dt)
        if h is None:
            g = self.groups[dt]
            h = self._result_host[dt] = torch.empty(max(g.length, 1), dtype=g.out_dtype).pin_memory()
        return h

    def _chunk_plan(self, dt: torch.dtype, chunks: int):
        """[(lo, hi, pointer table at column lo, host scatter plan)] for the
        group's columns in ``chunks`` ranges (bounds at multiples of 64K
        elements, so every range start stays 16-byte aligned).  Cached."""
        key = (dt, chunks)
        plan = self._plans.get(key)
        if plan is not None:
            return plan
        g = self.groups[dt]
        L = g.length
        step = max(1, -(-L // max(1, chunks)))
        step = (step + 65535) // 65536 * 65536
        bounds = [(lo, min(L, lo + step)) for lo in range(0, L, step)] or [(0, 0)]
        offs = np.array(g.offsets, dtype=np.int64)
        ends = offs + np.array(g.numels, dtype=np.int64)
        oesz = torch.empty((), dtype=g.out_dtype).element_size()
        plan = []
        for lo, hi in bounds:
            d_ptrs = g.d_ptrs + lo * g.esize
            s = np.maximum(offs, lo)
            e = np.minimum(ends, hi)
            idx = np.nonzero(e > s)[0]
            plan.append((lo, hi, d_ptrs, (idx, np.ascontiguousarray(s[idx] * oesz),
                                          np.ascontiguousarray((s[idx] - offs[idx]) * oesz),
                                          np.ascontiguousarray((e[idx] - s[idx]) * oesz))))
        self._plans[key] = plan
        return plan

    def _host_results(self, into: Optional[Dict[str, torch.Tensor]]) -> Dict[str, torch.Tensor]:
        per_key = {}
        for g in self.groups.values():
            for key, shape in zip(g.keys, g.shapes):
                t = into.get(key) if into is not None else None
                if t is None or t.dtype != g.out_dtype or not t.is_contiguous() or t.is_cuda \
                        or tuple(t.shape) != tuple(shape):
                    t = torch.empty(shape, dtype=g.out_dtype)
                per_key[key] = t
        return per_key

    def _unpack_group(self, g, h: torch.Tensor, per_key: Dict[str, torch.Tensor]) -> None:
        esz = h.element_size()
        ts, offs, nbytes = [], [], []
        for key, off, n in zip(g.keys, g.offsets, g.numels):
            if n:
                ts.append(per_key[key].data_ptr())
                offs.append(off * esz)
                nbytes.append(n * esz)
        n = len(ts)
        if n:
            nat.check(nat.lib().fedagg_host_unpack(h.data_ptr(), (ctypes.c_void_p * n)(*ts),
                                                   (ctypes.c_int64 * n)(*offs), (ctypes.c_int64 * n)(*nbytes),
                                                   n, _PACK_THREADS), "host_unpack")

    def _take_result_pool(self) -> Optional[Dict[str, torch.Tensor]]:
        th = self._pool_thread
        if th is None:
            return None
        th.join()
        self._pool_thread = None
        pool, self._pool = self._pool, None
        return pool

    def _refill_result_pool(self) -> None:
        """Allocate and touch the next call's per-key host tensors on a
        background thread (torch releases the GIL inside the fills)."""
        import threading

        shapes = [(k, s, g.out_dtype) for g in self.groups.values() for k, s in zip(g.keys, g.shapes)]

        def work():
            pool = {}
            for k, s, dt in shapes:
                pool[k] = torch.zeros(s, dtype=dt)
            self._pool = pool

        self._pool_thread = threading.Thread(target=work, name="fedagg-result-pool", daemon=True)
        _POOL_THREADS.add(self._pool_thread)
        self._pool_thread.start()


# pool threads still filling at interpreter exit are joined first (a daemon
# thread inside a torch op during finalisation can crash the exit)
_POOL_THREADS: "weakref.WeakSet" = weakref.WeakSet()


@atexit.register
def _join_pool_threads() -> None:
    for th in list(_POOL_THREADS):
        th.join()

