"""One round's client updates spread over several GPUs of ONE server process.

FedML's server is a single process (python/fedml/__init__.py:330-348 forces
``n_proc_in_silo = 1`` for it), and every client update reaches that process
(cross_silo/server/fedml_aggregator.py:58-67).  When a round does not fit one
MI355X (512 clients x a 300M-parameter bf16 model is 311 GB), or when the
caller lists several devices (``args.fedagg_devices``), the round is cut along
the PARAMETER axis inside the process:

* **Whole keys per device.**  The state dict's keys are dealt to G devices by
  bytes, largest first, each to the least-loaded device (LPT), and every
  device holds an ordinary ``ClientBucket`` over its keys, in the model's key
  order.  A key never straddles two devices, so a client's dict can be
  rebound to views that are ordinary one-device tensors (the cross-silo
  mirror does that on arrival, as the reference moves tensors to its server
  device), and the result of every key is an ordinary tensor.  The balance
  cost is bounded by the largest key; after LPT a local search moves or
  swaps keys between the heaviest device and the others.  The heaviest
  device's excess over the mean (tests/test_multidev.py): ResNet-50 under
  0.001 % on 2, 4 and 8 devices; ViT-B/16 0.84 % on 4 and 3.6 % on 8 (its
  2.36M-element MLP matrices are 2.7 % of the model each); config 5's 128
  equal LoRA keys exact on 2, 4 and 8.
* **Ingest.**  ``put`` sends each device its keys from the arriving dict: one
  pinned pack + one async H2D per device and dtype, on that device's own copy
  stream and PCIe link.  Every device's staging row of the arriving client is
  packed in ONE native gather (fedagg_host_gather, a persistent thread pool),
  then the G H2Ds are issued back to back, so G links carry a client at once.
* **Reduction.**  Every device runs the single-GPU kernels over its keys in
  the reference's client order: no exchange and bit-exact with one GPU.
  ``reduce_to_host`` enqueues every device's reductions and D2H copies before
  waiting for any, then scatters each device's result into the per-key host
  tensors.

Several shards may sit on the same device (tests run G = 2 and 4 shards on a
one-GPU box); each is then its own bucket on that device.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as nat
from . import kernels as kn
from .bucket import ClientBucket, _pad, gather_jobs
from .layout import INT_DTYPES, numel

_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _raw_stream(device: torch.device) -> int:
    """torch's current stream on `device` as a raw hipStream_t."""
    if _RAW_STREAM is not None:
        return _RAW_STREAM(device.index)
    return torch.cuda.current_stream(device).cuda_stream


Entry = Tuple[str, Tuple[int, ...], torch.dtype]

# row bytes per element of each storage dtype (integer keys go into fp32 rows
# when promoted, int64 rows otherwise)
_ROW_ESZ = {torch.float32: 4, torch.bfloat16: 2, torch.float16: 2, torch.float64: 8, torch.int64: 8}
_CODE = {torch.float32: nat.DT_F32, torch.bfloat16: nat.DT_BF16, torch.float16: nat.DT_F16,
         torch.float64: nat.DT_F64, torch.int64: nat.DT_I64}


def _entries(layout) -> List[Entry]:
    if isinstance(layout, dict):
        return [(k, tuple(t.shape), t.dtype) for k, t in layout.items()]
    return [(k, tuple(s), d) for k, s, d in layout]


def entry_bytes(entry: Entry, promote_ints: bool = True) -> int:
    """Row bytes one client's key occupies."""
    _, shape, dt = entry
    if dt in INT_DTYPES:
        dt = torch.float32 if promote_ints else torch.int64
    return numel(shape) * _ROW_ESZ.get(dt, 8)


def _refine(sizes: List[int], owner: List[int], load: List[int], rounds: int = 512) -> None:
    """Local search after LPT: move one key from the most loaded device to
    another, or swap two keys between them, while that lowers the heavier
    of the pair below the current maximum.  Deterministic; stops when no
    move or swap helps."""
    G = len(load)
    if G < 2:
        return
    for _ in range(rounds):
        hi = max(range(G), key=lambda s: (load[s], -s))
        on_hi = [i for i, o in enumerate(owner) if o == hi and sizes[i]]
        best = None  # (new max of the pair, i, lo, j or -1)
        for lo in range(G):
            gap = load[hi] - load[lo]
            if lo == hi or gap <= 0:
                continue
            on_lo = [j for j, o in enumerate(owner) if o == lo and sizes[j]]
            for i in on_hi:
                if sizes[i] < gap:
                    m = max(load[hi] - sizes[i], load[lo] + sizes[i])
                    if best is None or m < best[0]:
                        best = (m, i, lo, -1)
                for j in on_lo:
                    d = sizes[i] - sizes[j]
                    if 0 < d < gap:
                        m = max(load[hi] - d, load[lo] + d)
                        if best is None or m < best[0]:
                            best = (m, i, lo, j)
        if best is None or best[0] >= load[hi]:
            return
        _, i, lo, j = best
        owner[i] = lo
        load[hi] -= sizes[i]
        load[lo] += sizes[i]
        if j >= 0:
            owner[j] = hi
            load[lo] -= sizes[j]
            load[hi] += sizes[j]


def shard_plan(layout, shards: int, promote_ints: bool = True) -> List[List[Entry]]:
    """Deal whole keys to ``shards`` devices by bytes: largest first, each to
    the least-loaded device (ties to the lowest index); inside a device the
    keys keep the model's order.  Empty keys go to device 0.  Devices that
    receive nothing are dropped (more devices than keys with data)."""
    entries = _entries(layout)
    if shards < 1:
        raise ValueError("shards must be >= 1")
    sizes = [entry_bytes(e, promote_ints) for e in entries]
    load = [0] * shards
    owner = [0] * len(entries)
    for i in sorted(range(len(entries)), key=lambda i: (-sizes[i], i)):
        if sizes[i] == 0:
            continue
        g = min(range(shards), key=lambda s: (load[s], s))
        owner[i] = g
        load[g] += sizes[i]
    _refine(sizes, owner, load)
    out: List[List[Entry]] = [[] for _ in range(shards)]
    for e, g in zip(entries, owner):
        out[g].append(e)
    keep = [s for g, s in enumerate(out) if g == 0 or any(entry_bytes(e, promote_ints) for e in s)]
    return keep


def shard_loads(plan: Sequence[Sequence[Entry]], promote_ints: bool = True) -> List[int]:
    return [sum(entry_bytes(e, promote_ints) for e in s) for s in plan]


def merge_in_order(entries: Sequence[Entry], parts: Sequence[Dict[str, torch.Tensor]]
                   ) -> "OrderedDict[str, torch.Tensor]":
    """Reassemble per-device results into one dict in the model's key order."""
    res = OrderedDict()
    for key, _, _ in entries:
        for p in parts:
            if key in p:
                res[key] = p[key]
                break
        else:
            raise KeyError(key)
    return res


def split_tables(entries: Sequence[Entry], plan: Sequence[Sequence[Entry]], tables: Dict[int, np.ndarray]
                 ) -> List[Dict[int, np.ndarray]]:
    """The native walker's host pointer tables ({code: int64 [T_code, K]},
    rows = the keys of that dtype in the model's order) cut into one table
    per device, rows in that device's key order (what ClientBucket.
    put_from_table / put_batch read)."""
    code_of = {k: _CODE.get(d) for k, _, d in entries}
    row_of: Dict[str, int] = {}
    count: Dict[int, int] = {}
    for k, _, d in entries:
        c = code_of[k]
        if c is None or c not in tables:
            continue
        row_of[k] = count.get(c, 0)
        count[c] = row_of[k] + 1
    out = []
    for shard in plan:
        sub: Dict[int, List[int]] = {}
        for k, _, _ in shard:
            if k in row_of:
                sub.setdefault(code_of[k], []).append(row_of[k])
        out.append({c: np.ascontiguousarray(tables[c][rows]) for c, rows in sub.items()})
    return out


def parse_devices(spec) -> List[torch.device]:
    """``args.fedagg_devices``: "all", "0,1,2", [0, 1], ["cuda:0", "cuda:1"]
    or torch.devices.  A device may repeat (several shards on one GPU)."""
    if spec is None:
        return []
    if isinstance(spec, str):
        if spec.strip() == "all":
            return [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
        spec = [s.strip() for s in spec.split(",") if s.strip()]
    out = []
    for s in spec:
        if isinstance(s, torch.device):
            d = s
        elif isinstance(s, int) or (isinstance(s, str) and s.isdigit()):
            d = torch.device("cuda", int(s))
        else:
            d = torch.device(s)
        if d.type != "cuda":
            raise ValueError(f"fedagg_devices: {s!r} is not a CUDA device")
        if d.index is None:
            d = torch.device("cuda", 0)
        out.append(d)
    return out


def round_bytes(layout, capacity: int, promote_ints: bool = True) -> int:
    """HBM a one-device ClientBucket of this round takes (rows + results)."""
    per_dt: Dict[torch.dtype, int] = {}
    for e in _entries(layout):
        dt = e[2]
        if dt in INT_DTYPES:
            dt = torch.float32 if promote_ints else torch.int64
        per_dt[dt] = per_dt.get(dt, 0) + numel(e[1]) + 8
    return sum((capacity + 1) * _pad(n) * _ROW_ESZ.get(dt, 8) for dt, n in per_dt.items())


def visible_devices() -> List[torch.device]:
    """Every GPU this process sees (the devices an over-HBM round spreads to)."""
    return [torch.device("cuda", i) for i in range(torch.cuda.device_count())]


def free_bytes(device: torch.device) -> int:
    """HBM a new round can take on ``device``: the driver's free memory plus
    what torch's caching allocator holds reserved but unused (freed blocks it
    would hand out again before asking the driver)."""
    free, _ = torch.cuda.mem_get_info(device)
    try:
        free += max(0, torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device))
    except (RuntimeError, AssertionError):
        pass
    return free


def devices_for_round(args, layout, capacity: int, default: torch.device, promote_ints: bool = True
                      ) -> List[torch.device]:
    """Where a round's bucket goes: ``args.fedagg_devices`` when it lists
    devices; otherwise every visible GPU when the round does not fit the
    default device's free HBM (``free_bytes``, with 10 % headroom) and more
    GPUs exist; otherwise just the default device.  Callers decide once per
    round layout (a resident bucket is not free memory any more; see
    agg_operator._round_devices and the cross-silo mirror's first update)."""
    devs = parse_devices(getattr(args, "fedagg_devices", None)) if args is not None else []
    if devs:
        return devs
    if torch.cuda.device_count() > 1:
        if round_bytes(layout, capacity, promote_ints) > 0.9 * free_bytes(default):
            return visible_devices()
    return [default]


class MultiDeviceBucket:
    """A round's client updates over G devices, whole keys per device
    (``shard_plan``).  Same ingest / reduce interface as ClientBucket."""

    def __init__(self, layout, capacity: int, devices: Sequence, low_precision_acc: str = "reference",
                 promote_ints: bool = True):
        devices = [torch.device(d) for d in devices]
        if not devices:
            raise ValueError("MultiDeviceBucket needs at least one device")
        self.entries = _entries(layout)
        self.capacity = capacity
        self.promote_ints = promote_ints
        self.plan = shard_plan(self.entries, len(devices), promote_ints)
        self.devices = devices[:len(self.plan)]
        self.shards: List[ClientBucket] = [
            ClientBucket(sub, capacity, dev, low_precision_acc=low_precision_acc, promote_ints=promote_ints)
            for sub, dev in zip(self.plan, self.devices)]
        self.owner: Dict[str, int] = {k: g for g, sub in enumerate(self.plan) for k, _, _ in sub}
        self.sample_nums: List[Optional[float]] = [None] * capacity
        self.int_keys = set().union(*(b.int_keys for b in self.shards))
        self.acc_mode = self.shards[0].acc_mode
        self.entry_keys = [k for k, _, _ in self.entries]
        self._slot_dicts: Dict[int, tuple] = {}
        self._slot_of: Dict[int, int] = {}

    # ---- ingest ---------------------------------------------------------------

    def put(self, slot: int, state_dict, sample_num: float) -> None:
        """One client: every device takes its keys (device tensors D2D; host
        keys packed into each device's pinned staging row, ALL devices' rows
        in one native gather, then one H2D per device and dtype on its own
        copy stream, issued back to back so the G links carry the client at
        once)."""
        jobs = [(b, b.put_prepare(slot, state_dict, sample_num)) for b in self.shards]
        gather_jobs([j for _, js in jobs for j in js])
        for b, js in jobs:
            b.put_issue(js)
        self.sample_nums[slot] = sample_num

    def split_tables(self, tables: Dict[int, np.ndarray]) -> List[Dict[int, np.ndarray]]:
        return split_tables(self.entries, self.plan, tables)

    def put_from_tables(self, slot: int, shard_tables: Sequence[Dict[int, np.ndarray]], state_dict,
                        sample_num: float) -> None:
        """put() for one client of a walked host round (``split_tables`` of
        the walker's tables, computed once per round)."""
        jobs = [(b, b.put_from_table_prepare(slot, t, state_dict, sample_num))
                for b, t in zip(self.shards, shard_tables)]
        gather_jobs([j for _, js in jobs for j in js])
        for b, js in jobs:
            b.put_issue(js)
        self.sample_nums[slot] = sample_num

    def put_batch(self, shard_tables: Sequence[Dict[int, np.ndarray]], state_dicts, sample_nums) -> None:
        for b, t in zip(self.shards, shard_tables):
            b.put_batch({c: np.ascontiguousarray(a).ravel() for c, a in t.items()}, state_dicts, sample_nums)
        for i, n in enumerate(sample_nums):
            self.sample_nums[i] = n

    def sync_ingest(self) -> None:
        for b in self.shards:
            b.sync_ingest()

    def wait_ingest(self) -> None:
        for b in self.shards:
            b.wait_ingest()

    def view(self, slot: int) -> "OrderedDict[str, torch.Tensor]":
        """Views of slot's row on each key's device, in the model's key order."""
        return merge_in_order(self.entries, [b.view(slot) for b in self.shards])

    # ---- reduction ------------------------------------------------------------

    def weights(self, sample_nums: Sequence[float]) -> List[float]:
        return self.shards[0].weights(sample_nums)

    def aggregate(self, sample_nums: Optional[Sequence[float]] = None, num_clients: Optional[int] = None
                  ) -> "OrderedDict[str, torch.Tensor]":
        """FedAvg over the first K slots; every key's result on its device
        (each device's launches go on that device's current stream)."""
        K = num_clients if num_clients is not None else self.capacity
        ns = list(sample_nums) if sample_nums is not None else self.sample_nums[:K]
        if any(n is None for n in ns):
            raise ValueError("sample count missing for some slot")
        w = self.weights(ns)
        outs_list = [b.new_outputs() for b in self.shards]
        if not self.reduce_into_all(outs_list, w, K):
            for b, outs in zip(self.shards, outs_list):
                with torch.cuda.device(b.device):
                    b.reduce_into(outs, w, K)
        return merge_in_order(self.entries, [b.unflatten(o) for b, o in zip(self.shards, outs_list)])

    def reduce_into_all(self, outs_list: Sequence[Dict[torch.dtype, torch.Tensor]], weights: Sequence[float],
                        num_clients: Optional[int] = None, events: Optional[Sequence] = None,
                        slots: Optional[Sequence[int]] = None) -> bool:
        """Every device's reduction in ONE native call (fedagg_wsum_fedopt_batch
        with FEDAGG_FEDOPT_AVG launches, each on its device's current stream),
        so the last device starts one launch after the one before it instead
        of one Python reduce_into later.  The arithmetic is each shard's
        reduce_into's (the same kernels, the same bits).  events[s]: optional
        (start, end) torch.cuda.Events around shard s's launch.  Returns False
        and launches nothing when a shard needs more than one launch (several
        dtype groups) or K > 256 (weights not by value); the caller then uses
        the shards' reduce_into."""
        K = num_clients if num_clients is not None else (len(slots) if slots is not None else self.capacity)
        if slots is not None and (len(slots) != K or any(not 0 <= s < self.capacity for s in slots)):
            raise ValueError("slots: one valid slot per client")
        if not 1 <= K <= self.capacity and slots is None:
            raise ValueError(f"num_clients {K} outside [1, {self.capacity}]")
        if len(weights) != K:
            raise ValueError("one weight per client")
        if K > kn.INLINE_MAX_K:
            return False
        groups = []
        for b in self.shards:
            live = [(dt, g) for dt, g in b.groups.items() if g.length]
            if len(live) > 1:
                return False
            groups.append(live[0] if live else None)
        if slots is not None and list(slots) == list(range(K)):
            slots = None
        tabs = [b.slot_ptrs(slots) if slots is not None else None for b in self.shards]
        key = tuple((o[dg[0]].data_ptr() if dg else 0, t[dg[0]].data_ptr() if (dg and t is not None) else 0)
                    for o, dg, t in zip(outs_list, groups, tabs))
        cache = getattr(self, "_avg_table", None)
        if cache is None or cache[0] != key or cache[2] != K:
            n = sum(1 for dg in groups if dg is not None)
            tab = (nat.FedOptLaunch * n)()
            i = 0
            for b, o, dg, t in zip(self.shards, outs_list, groups, tabs):
                if dg is None:
                    continue
                dt, g = dg
                d = tab[i]
                d.d_src = (g.d_ptrs if t is None else t[dt]).data_ptr()
                d.d_param = o[dt].data_ptr()
                d.N, d.K, d.opt, d.device = g.length, K, nat.FEDOPT_AVG, b.device.index
                d.dtype, d.acc_mode = _CODE[dt], b.acc_mode
                d.flags = nat.FEDAGG_HOST_WEIGHTS | (nat.FEDAGG_ALIGNED16 if (o[dt].data_ptr() & 15) == 0 else 0)
                i += 1
            cache = self._avg_table = (key, tab, K)
        tab = cache[1]
        w32 = kn.weights_for(weights, torch.float32, self.devices[0])
        w64 = kn.weights_for(weights, torch.float64, self.devices[0]) if any(
            dg is not None and dg[0] == torch.float64 for dg in groups) else None
        i = 0
        live = []
        for s, (b, dg) in enumerate(zip(self.shards, groups)):
            if dg is None:
                continue
            b.sync_ingest()
            stream = _raw_stream(b.device)
            d = tab[i]
            d.weights = (w64 if dg[0] == torch.float64 else w32).data_ptr()
            d.stream = stream
            live.append((s, b))
            i += 1
        if events is not None:
            for s, b in live:
                if events[s] is not None:
                    events[s][0].record(torch.cuda.current_stream(b.device))
        if len(tab):
            nat.check(nat.lib().fedagg_wsum_fedopt_batch(tab, len(tab)), "multi-device reduction")
        if events is not None:
            for s, b in live:
                if events[s] is not None:
                    events[s][1].record(torch.cuda.current_stream(b.device))
        if slots is not None:  # the slot tables were read on these streams
            for (s, b), t in zip(live, [tabs[s] for s, _ in live]):
                t[groups[s][0]].record_stream(torch.cuda.current_stream(b.device))
        return True

    def bind_slot(self, slot: int, state_dict, view) -> None:
        """As ClientBucket.bind_slot: state_dict's values are now ``view``'s
        (this slot's views on their keys' devices)."""
        old = self._slot_dicts.get(slot)
        if old is not None:
            self._slot_of.pop(id(old[0]), None)
        self._slot_dicts[slot] = (state_dict, view)
        self._slot_of[id(state_dict)] = slot

    def reduce_slots(self, slots: Sequence[int], weights: Sequence[float]) -> "OrderedDict[str, torch.Tensor]":
        """FedAvg of the given slots on every device (each device's launches
        enqueued before the next device's), results on their keys' devices
        in the model's key order."""
        outs_list = [b.new_outputs() for b in self.shards]
        if not self.reduce_into_all(outs_list, weights, len(slots), slots=slots):
            return merge_in_order(self.entries, [b.reduce_slots(slots, weights) for b in self.shards])
        return merge_in_order(self.entries, [b.unflatten(o) for b, o in zip(self.shards, outs_list)])

    def reduce_to_host(self, weights: Sequence[float], num_clients: Optional[int] = None,
                       into: Optional[Dict[str, torch.Tensor]] = None, chunks: int = 8
                       ) -> "OrderedDict[str, torch.Tensor]":
        """The averaged model as independent host tensors: every device's
        reductions and D2H copies are enqueued before any is waited for, then
        each device's result is scattered into the per-key tensors."""
        states = [b.launch_to_host(weights, num_clients, into, chunks) for b in self.shards]
        parts = [b.finish_to_host(s) for b, s in zip(self.shards, states)]
        return merge_in_order(self.entries, parts)

    # ---- accounting -----------------------------------------------------------

    def algorithmic_bytes(self, num_clients: Optional[int] = None) -> int:
        return sum(b.algorithmic_bytes(num_clients) for b in self.shards)

    def shard_bytes(self) -> List[int]:
        return shard_loads(self.plan, self.promote_ints)

    def num_elements(self) -> int:
        return sum(b.num_elements() for b in self.shards)
