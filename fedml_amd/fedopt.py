"""FedOpt server aggregation on MI355X: FedAvg fused with the server optimizer.

Mirrors the server side of python/fedml/simulation/mpi/fedopt/FedOptAggregator.py
(the reference's working FedOpt path; the plugin operator's "FedOpt" branch is
`pass`, agg_operator.py:64-65):

  add_local_trained_result(index, model_params, sample_num)   :68-72
  check_whether_all_receive()                                  :74-80
  aggregate()                                                  :81-116
      FedAvg of the round (:93-101), then for every NAMED PARAMETER
      grad = p_old - p_avg (:118-125) and one torch.optim.<server_optimizer>
      step with lr=server_lr, momentum=server_momentum (:49-54, :104-112);
      buffers (BatchNorm running stats, num_batches_tracked) take the
      average, int64 ones truncated by load_state_dict's copy_ (:126-130).

Supported server optimizers (OptRepo names, optrepo.py:10); parameters are fp32:
  "sgd"   with or without momentum — what the MPI aggregator builds (it passes
          `momentum=` to the constructor, :49-54).
  "adam"  torch.optim.Adam with its defaults and lr=server_lr, as the SP
          FedOptAPI builds it (sp/fedopt/fedopt_api.py:78-85; the MPI aggregator
          cannot: Adam rejects `momentum=`).  server_momentum is ignored.  The
          step is fused like SGD's (fedagg_wsum_fedopt_adam_f32); exp_avg and
          exp_avg_sq are bit-identical to torch's CPU Adam, the parameters
          differ only where torch's CPU sqrt is not correctly rounded
          (tests/test_gpu_fedopt.py).
  "adagrad" torch.optim.Adagrad with its defaults (lr_decay 0, eps 1e-10,
          initial_accumulator_value 0) and lr=server_lr, the SP FedOptAPI's
          construction again (FedAdagrad).  Fused like Adam's
          (fedagg_wsum_fedopt_adagrad_f32); state_sum is bit-identical to
          torch's, parameters carry the same sqrt caveat.
  "adamw" torch.optim.AdamW with its defaults (betas (0.9, 0.999), eps 1e-8,
          weight_decay 0.01 unless server_weight_decay says otherwise):
          Adam with the parameter scaled by fl32(1 - lr*wd) first
          (fedagg_wsum_fedopt_adamw_f32); moments bit-identical to torch,
          parameters with Adam's sqrt caveat.
  "rmsprop" torch.optim.RMSprop with its defaults (alpha 0.99, eps 1e-8,
          momentum 0, not centered, weight_decay 0)
          (fedagg_wsum_fedopt_rmsprop_f32); square_avg bit-identical to
          torch, parameters with the sqrt caveat.
  "adamax" / "nadam" / "radam" / "adadelta" / "asgd" / "rprop"
          the other elementwise optimizers OptRepo names, with torch's
          defaults and lr=server_lr as FedOptAPI builds them
          (fedagg_wsum_fedopt_optrepo_f32, the per-element rules beside
          OptRepoEpi in csrc/fedagg.hip).  Adamax, ASGD and Rprop take no
          sqrt and are bit-exact with torch, state included; NAdam, RAdam and
          Adadelta carry Adam's sqrt caveat (Adadelta's acc_delta too, since
          it is built from a square root).  server_momentum is ignored for
          them, as for Adam.
Any other OptRepo name (LBFGS needs a closure, SparseAdam sparse gradients,
Adafactor and Muon are not elementwise), and weight decay / momentum /
centered variants of these, raise NotImplementedError.

A client dict added at two indices (add_local_trained_result) behaves as in
FedOptAggregator.aggregate (:93-101): the averaged dict IS index 0's, so an
index holding that same dict object reads the running average at its turn
in the loop.  Such a round is reduced by the aliasing program of
fedml_amd.agg_operator (_run_cells) and then stepped with the average as one
source at weight 1.0, bit-identical to the reference's chain.

Device layout: the round's updates sit in a ClientBucket; the global model
and the momentum buffers are flat fp32 vectors with the bucket's fp32 layout.
Every maximal run of consecutive parameter keys is ONE fused launch
(fedagg_wsum_fedopt_sgd_f32: the average never reaches HBM), every run of
buffer keys one plain FedAvg launch writing straight into the global vector.
For a LoRA adapter set (config 5) all keys are parameters: one launch.
"""
from __future__ import annotations

from collections import OrderedDict
import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _native as nat
from . import kernels as kn
from .bucket import ClientBucket

_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _raw_stream(device: torch.device) -> int:
    """torch's current stream on `device` as a raw hipStream_t."""
    if _RAW_STREAM is not None:
        return _RAW_STREAM(device.index)
    return torch.cuda.current_stream(device).cuda_stream

# the OptRepo optimizers of fedagg_wsum_fedopt_optrepo_f32 and their
# per-element state buffers (torch's state names, in the kernel's order)
OPTREPO_STATE = {"adamax": ("exp_avg", "exp_inf"), "nadam": ("exp_avg", "exp_avg_sq"),
                 "radam": ("exp_avg", "exp_avg_sq"), "adadelta": ("square_avg", "acc_delta"),
                 "asgd": ("ax",), "rprop": ("prev", "step_size")}
FUSED_OPTIMIZERS = ("sgd", "adam", "adamw", "adagrad", "rmsprop") + tuple(OPTREPO_STATE)
# OptRepo names that cannot be a fused elementwise server step
_NOT_ELEMENTWISE = {"lbfgs": "torch.optim.LBFGS.step() needs a closure",
                    "sparseadam": "torch.optim.SparseAdam takes sparse gradients only",
                    "adafactor": "torch.optim.Adafactor's second moment is factored over rows and columns",
                    "muon": "torch.optim.Muon orthogonalises 2-D updates (Newton-Schulz matrix products)"}


def _unsupported(name: str) -> NotImplementedError:
    why = _NOT_ELEMENTWISE.get(name.lower())
    return NotImplementedError(f"server_optimizer {name!r}: " + (f"{why}; " if why else "") +
                               f"{FUSED_OPTIMIZERS} are fused")


def optrepo_carry(optimizer: str, lr: float) -> "ctypes.Array":
    """The fp32 scalar state of an OptRepo optimizer before its first step:
    NAdam's mu_product 1.0; ASGD's eta fl32(lr) and mu 1.0."""
    import ctypes

    c = (ctypes.c_float * 2)()
    if optimizer == "nadam":
        c[0] = 1.0
    elif optimizer == "asgd":
        c[0], c[1] = lr, 1.0
    return c


def _ref(obj):
    """A reference that does not keep a client's dict alive where Python
    allows it (OrderedDict, every state_dict), a strong one otherwise."""
    import weakref

    try:
        return weakref.ref(obj)
    except TypeError:
        return lambda: obj


def _weight_decay(optimizer: str, weight_decay: Optional[float]) -> float:
    """torch's default weight decay of each fused optimizer; AdamW's is the
    only one the fused steps apply (decoupled), the others must stay 0."""
    if optimizer == "adamw":
        return 0.01 if weight_decay is None else float(weight_decay)
    if weight_decay:
        raise NotImplementedError(f"server_optimizer {optimizer!r} with weight_decay={weight_decay}: not fused")
    return 0.0


def _check_momentum(optimizer: str, momentum) -> None:
    """torch.optim.RMSprop takes `momentum=` and applies it (a momentum buffer
    over g / (sqrt(v) + eps)); the MPI FedOptAggregator passes
    server_momentum to the constructor (FedOptAggregator.py:49-54), so an
    RMSprop server with momentum is a different optimizer from the fused one.
    Refuse it rather than silently dropping the momentum.  Adam / AdamW /
    Adagrad have no `momentum` argument (torch raises TypeError there; the SP
    FedOptAPI passes lr only, fedopt_api.py:78-85), so it is ignored for them."""
    if optimizer == "rmsprop" and momentum:
        raise NotImplementedError(f"server_optimizer 'rmsprop' with server_momentum={momentum}: only the "
                                  "momentum-free RMSprop step is fused")


class FedOptServer:
    def __init__(self, global_state: "OrderedDict[str, torch.Tensor]", param_names: Sequence[str],
                 worker_num: int, server_optimizer: str = "sgd", server_lr: float = 1.0,
                 server_momentum: float = 0.0, device=None, server_weight_decay: Optional[float] = None):
        self.optimizer = server_optimizer.lower()
        if self.optimizer not in FUSED_OPTIMIZERS:
            raise _unsupported(server_optimizer)
        self.lr = float(server_lr)
        _check_momentum(self.optimizer, server_momentum)
        self.momentum = float(server_momentum) if self.optimizer == "sgd" else 0.0
        # torch.optim defaults (sp/fedopt/fedopt_api.py:79-85 passes lr only)
        self.betas, self.eps = (0.9, 0.999), (1e-10 if self.optimizer == "adagrad" else 1e-8)
        self.alpha = 0.99  # RMSprop
        self.weight_decay = _weight_decay(self.optimizer, server_weight_decay)
        self.lr_decay = 0.0
        self.step_count = 0
        self.worker_num = worker_num
        self.param_names = list(param_names)
        self.bucket = ClientBucket(global_state, worker_num, device)
        self.device = self.bucket.device
        for k in self.param_names:
            if global_state[k].dtype != torch.float32:
                raise TypeError(f"parameter {k!r} is {global_state[k].dtype}; the fused server step is fp32")
        f32 = self.bucket.groups.get(torch.float32)
        with torch.cuda.device(self.device):
            self.global_flat: Dict[torch.dtype, torch.Tensor] = self.bucket.new_outputs()
            self._int_state: "OrderedDict[str, torch.Tensor]" = OrderedDict()
            # the global model in the bucket's flat layout; integer buffers
            # (num_batches_tracked) also keep their own tensor of their dtype
            for k, t in global_state.items():
                g, j = self.bucket.where[k]
                self.global_flat[g.dtype][g.offsets[j]:g.offsets[j] + g.numels[j]].copy_(t.detach().reshape(-1))
                if k in self.bucket.int_keys:
                    self._int_state[k] = t.detach().to(self.device).clone()
            self.mom = torch.zeros_like(self.global_flat[torch.float32]) if (f32 and self.momentum) else None
            adam = f32 and self.optimizer in ("adam", "adamw")
            self.exp_avg = torch.zeros_like(self.global_flat[torch.float32]) if adam else None
            self.exp_avg_sq = torch.zeros_like(self.global_flat[torch.float32]) if adam else None
            # Adagrad's state_sum, RMSprop's square_avg: both start at zero
            acc = f32 and self.optimizer in ("adagrad", "rmsprop")
            self.state_sum = torch.zeros_like(self.global_flat[torch.float32]) if acc else None
            # the OptRepo optimizers' per-element state, as torch creates it
            self.opt_state: Dict[str, torch.Tensor] = {}
            if f32 and self.optimizer in OPTREPO_STATE:
                for name in OPTREPO_STATE[self.optimizer]:
                    self.opt_state[name] = torch.zeros_like(self.global_flat[torch.float32])
                if self.optimizer == "rprop":  # step_size = full_like(grad, lr)
                    self.opt_state["step_size"].fill_(self.lr)
        self._carry = optrepo_carry(self.optimizer, self.lr)
        self.first_step = True
        self._views: Optional["OrderedDict[str, torch.Tensor]"] = None
        self.runs: List[Tuple[bool, int, int]] = self._runs(f32) if f32 else []
        self.run_ptrs = [kn.upload_i64([f32.rows[i].data_ptr() + lo * 4 for i in range(worker_num)], self.device)
                         for _, lo, _ in self.runs]
        self.model_dict: Dict[int, "OrderedDict"] = {}
        self.sample_num_dict: Dict[int, float] = {}
        self.flag_client_model_uploaded_dict = {i: False for i in range(worker_num)}
        self._refs: Dict[int, object] = {}  # index -> reference to the dict added there this round
        self._same: set = set()  # {i, j} index pairs that were handed the same dict object

    def _runs(self, g) -> List[Tuple[bool, int, int]]:
        """Maximal runs of consecutive keys of one kind: (is_param, lo, hi)."""
        params = set(self.param_names)
        runs: List[Tuple[bool, int, int]] = []
        for key, off, n in zip(g.keys, g.offsets, g.numels):
            if n == 0:
                continue
            p = key in params
            if runs and runs[-1][0] == p:
                runs[-1] = (p, runs[-1][1], off + n)
            else:
                runs.append((p, off, off + n))
        return runs

    # ---- FedOptAggregator interface -----------------------------------------

    def add_local_trained_result(self, index: int, model_params, sample_num) -> None:
        """:68-72; the update goes straight into its HBM row."""
        self.bucket.put(index, model_params, sample_num)
        self.note_dict(index, model_params)
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

    def note_dict(self, index: int, model_params) -> None:
        """Remember which dict object index holds this round, and which other
        indices hold the same object (compared while both are alive, so a
        reused id() of a freed dict cannot match)."""
        self._same = {p for p in self._same if index not in p}
        for i, r in self._refs.items():
            if i != index and r() is model_params:
                self._same.add(frozenset((i, index)))
        self._refs[index] = _ref(model_params)

    def _aliases_of_client0(self) -> List[int]:
        """Indices j > 0 holding index 0's dict object: FedOptAggregator.py:
        93-101 reads the running average there."""
        return sorted(j for p in self._same if 0 in p for j in p if j != 0 and j < self.worker_num)

    def check_whether_all_receive(self) -> bool:
        for idx in range(self.worker_num):
            if not self.flag_client_model_uploaded_dict[idx]:
                return False
        for idx in range(self.worker_num):
            self.flag_client_model_uploaded_dict[idx] = False
        return True

    def aggregate(self, events=None) -> "OrderedDict[str, torch.Tensor]":
        """events: optional (start, end) torch.cuda.Events recorded around the
        fp32 launches (the benchmark's kernel timing)."""
        ns = [self.sample_num_dict[i] for i in range(self.worker_num)]
        weights = self.bucket.weights(ns)
        alias = self._aliases_of_client0()
        self._refs, self._same = {}, set()  # the round's dicts are consumed
        with torch.cuda.device(self.device):
            self.bucket.sync_ingest()
            if alias:
                return self._aggregate_aliased(ns, weights, alias, events)
            return self._step(self._table(), weights, events)

    # ---- the round's fused launches (fedagg_wsum_fedopt_batch) ---------------

    _OPT_CODE = {"sgd": nat.FEDOPT_SGD, "adam": nat.FEDOPT_ADAM, "adamw": nat.FEDOPT_ADAMW,
                 "adagrad": nat.FEDOPT_ADAGRAD, "rmsprop": nat.FEDOPT_RMSPROP, **nat.OPT_CODES}

    def _table(self, run_ptrs=None, K: Optional[int] = None):
        """The round's launch descriptors, one per run of parameter keys (the
        fused server step) or buffer keys (the plain FedAvg into the global
        vector), with every field that does not change between rounds filled
        in.  Cached for the bucket's own rows; `run_ptrs` / `K` build a
        one-off table over other sources (the aliased round's average)."""
        cached = run_ptrs is None
        if cached and getattr(self, "_launches", None) is not None:
            return self._launches
        run_ptrs = self.run_ptrs if run_ptrs is None else run_ptrs
        K = self.worker_num if K is None else K
        f32 = self.global_flat.get(torch.float32)
        if f32 is None or not self.runs:  # no fp32 keys: nothing fused (the other groups average in _after)
            tab = (nat.FedOptLaunch * 0)()
            if cached:
                self._launches, self._launches_keep = tab, (tab, [])
            return tab
        st = [None, None]
        if self.optimizer == "sgd":
            st = [self.mom, None]
        elif self.optimizer in ("adam", "adamw"):
            st = [self.exp_avg, self.exp_avg_sq]
        elif self.optimizer in ("adagrad", "rmsprop"):
            st = [self.state_sum, None]
        elif self.optimizer in OPTREPO_STATE:
            names = OPTREPO_STATE[self.optimizer]
            st = [self.opt_state[names[0]], self.opt_state[names[-1]] if len(names) > 1 else None]
        tab = (nat.FedOptLaunch * len(self.runs))()
        for d, (is_param, lo, hi), ptrs in zip(tab, self.runs, run_ptrs):
            d.d_src = ptrs.data_ptr()
            d.K, d.N = K, hi - lo
            d.d_param = f32.data_ptr() + 4 * lo
            d.opt = self._OPT_CODE[self.optimizer] if is_param else nat.FEDOPT_AVG
            if is_param:
                d.d_state0 = st[0].data_ptr() + 4 * lo if st[0] is not None else 0
                d.d_state1 = st[1].data_ptr() + 4 * lo if st[1] is not None else 0
            d.device = self.device.index
            d.lr, d.momentum, d.eps, d.alpha = self.lr, self.momentum, self.eps, self.alpha
            d.decay = 1 - self.lr * self.weight_decay  # ctypes rounds it to fp32, as torch does
            ptrs_all = [d.d_param] + ([d.d_state0, d.d_state1] if is_param else [])
            d.flags = nat.FEDAGG_ALIGNED16 if all((p & 15) == 0 for p in ptrs_all if p) else 0
        keep = (tab, list(run_ptrs))  # the tables stay alive as long as the descriptors point at them
        if cached:
            self._launches = tab
            self._launches_keep = keep
        return tab

    def _fill(self, tab, off: int, w32) -> None:
        """This round's fields of the descriptors tab[off : off + runs]: the
        weights, the step's scalars, the first-step flag, the stream."""
        step = self.step_count + 1
        scal = None
        if self.optimizer in ("adam", "adamw"):
            scal = kn.adam_scalars(self.lr, self.betas[0], self.betas[1], self.eps, step)
        elif self.optimizer in OPTREPO_STATE:
            scal = kn.optrepo_scalars(self.optimizer, self.lr, step, self._carry)
        self._scal = scal  # alive until the launch (host memory the launch reads)
        host_w = nat.FEDAGG_HOST_WEIGHTS if isinstance(w32, kn.HostWeights) else 0
        wptr = w32.data_ptr()
        sptr = ctypes.addressof(scal) if scal is not None else 0
        stream = _raw_stream(self.device)
        # torch's Adagrad: clr = lr / (1 + (step - 1) * lr_decay), in double
        clr = self.lr / (1 + (step - 1) * self.lr_decay) if self.optimizer == "adagrad" else None
        first = int(self.first_step)
        for i in range(off, off + len(self.runs)):
            d = tab[i]
            d.weights, d.scalars, d.stream, d.first_step = wptr, sptr, stream, first
            d.flags = (d.flags & nat.FEDAGG_ALIGNED16) | host_w
            if clr is not None:
                d.lr = clr

    def _after(self, weights, K: int, averaged=None) -> None:
        """The rest of a round after the fused launches: the other dtype
        groups' averages, the integer buffers' truncation, the step count."""
        for dt, g in self.bucket.groups.items():
            if dt == torch.float32 or g.length == 0:
                continue
            if averaged is not None:
                self.global_flat[dt][:g.length].copy_(averaged[dt][:g.length])
                continue
            w = kn.weights_for(weights, dt, self.device)
            kn.wsum_ptrs(dt, g.d_ptrs, w, K, g.length, self.global_flat[dt], True)
        for k, t in self._int_state.items():
            # load_state_dict's copy_: the float32 average truncates toward zero
            g, j = self.bucket.where[k]
            t.reshape(-1).copy_(self.global_flat[g.dtype][g.offsets[j]:g.offsets[j] + g.numels[j]])
        self.first_step = False
        self.step_count += 1

    def _step(self, tab, weights, events, K: Optional[int] = None, averaged=None
              ) -> "OrderedDict[str, torch.Tensor]":
        """One round's fused launches from a descriptor table (one native
        call, fedagg_wsum_fedopt_batch), then the rest of the round."""
        K = self.worker_num if K is None else K
        w32 = kn.weights_for(weights, torch.float32, self.device)  # by value for K <= 256
        if len(tab):
            self._fill(tab, 0, w32)
            if events is not None:
                events[0].record()
            nat.check(nat.lib().fedagg_wsum_fedopt_batch(tab, len(tab)), f"fedopt {self.optimizer} launches")
            if events is not None:
                events[1].record()
        self._after(weights, K, averaged)
        return self.get_global_model_params()

    def _aggregate_aliased(self, ns, weights, alias: List[int], events) -> "OrderedDict[str, torch.Tensor]":
        """A round whose index-0 dict was added again at `alias`: the
        reference's loop (FedOptAggregator.py:93-101) replayed over the
        bucket's rows by agg_operator._run_cells, which reads the running
        average wherever the loop reads index 0's dict again; then the
        optimizer steps from that average as ONE source at weight 1.0
        (fl(x * 1.0) = x: the same step bit for bit)."""
        from .agg_operator import _run_cells

        class _A:
            fedagg_low_precision_acc = "reference"
            fedagg_device = None

        views = [self.bucket.view(i) for i in range(self.worker_num)]
        raw = [(ns[i], views[i]) for i in range(self.worker_num)]
        for j in alias:
            raw[j] = (ns[j], views[0])
        keys = [k for k, _, _ in self.bucket.entries]
        _run_cells(raw, (1,), keys, weights, _A())
        avg = views[0]  # rebound to the round's average, key by key
        flat = self.bucket.new_outputs()
        for k in keys:
            g, j = self.bucket.where[k]
            flat[g.dtype][g.offsets[j]:g.offsets[j] + g.numels[j]].copy_(avg[k].reshape(-1))
        f32 = flat.get(torch.float32)
        run_ptrs = [kn.upload_i64([f32.data_ptr() + lo * 4], self.device) for _, lo, _ in self.runs] if f32 is not None \
            else []
        out = self._step(self._table(run_ptrs, 1), [1.0], events, K=1, averaged=flat)
        torch.cuda.current_stream(self.device).synchronize()  # the one-off tables and the flat average
        return out

    # ---- optimizer state (the reference's opt.state_dict() round trip) ------

    def _param_slices(self):
        for key in self.param_names:
            g, j = self.bucket.where[key]
            yield key, g.offsets[j], g.numels[j], g.shapes[j]

    def optimizer_state(self) -> Dict[str, object]:
        """Per named parameter, the state torch's optimizer would hold after the
        same rounds: {"step": n, <buffer>: {name: tensor}} with buffer
        "momentum_buffer" (sgd with momentum), "exp_avg" / "exp_avg_sq"
        (adam), "sum" (adagrad), "square_avg" (rmsprop) or OPTREPO_STATE's
        names, plus the fp32 scalar state as floats ("mu_product" for nadam,
        "eta" / "mu" for asgd; torch keeps one equal tensor per parameter).
        Copies; for checkpointing and parity checks."""
        out: Dict[str, object] = {"step": self.step_count}
        bufs = self._state_buffers()
        for name, flat in bufs.items():
            if flat is None or (self.step_count == 0 and self.optimizer != "adagrad"):
                continue
            out[name] = OrderedDict((k, flat[o:o + n].view(shape).clone()) for k, o, n, shape in self._param_slices())
        if self.step_count:  # the fp32 scalar state, the same for every parameter
            if self.optimizer == "nadam":
                out["mu_product"] = float(self._carry[0])
            elif self.optimizer == "asgd":
                out["eta"], out["mu"] = float(self._carry[0]), float(self._carry[1])
        return out

    def _state_buffers(self) -> Dict[str, Optional[torch.Tensor]]:
        """torch's per-parameter state names -> our flat buffers."""
        if self.optimizer == "sgd":
            return {"momentum_buffer": self.mom}
        if self.optimizer == "adagrad":
            return {"sum": self.state_sum}  # exists from construction in torch (initial_accumulator_value)
        if self.optimizer == "rmsprop":
            return {"square_avg": self.state_sum}  # created at the first step in torch
        if self.optimizer in OPTREPO_STATE:
            return {name: self.opt_state.get(name) for name in OPTREPO_STATE[self.optimizer]}
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}

    def load_optimizer_state(self, state: Dict[str, object]) -> None:
        """Inverse of optimizer_state() (resume, or the state a torch optimizer
        holds: the next aggregate() continues from it)."""
        step = int(state.get("step", 0))
        bufs = self._state_buffers()
        with torch.cuda.device(self.device):
            for name, flat in bufs.items():
                if flat is None:
                    continue
                src = state.get(name)
                if src is None:
                    if step:
                        raise KeyError(f"optimizer state at step {step} lacks {name!r}")
                    flat.zero_()  # a fresh optimizer's state
                    if name == "step_size":  # Rprop's starts at lr
                        flat.fill_(self.lr)
                    continue
                for k, o, n, _ in self._param_slices():
                    flat[o:o + n].copy_(src[k].detach().reshape(-1))
        self._carry = optrepo_carry(self.optimizer, self.lr)
        for i, name in enumerate({"nadam": ("mu_product",), "asgd": ("eta", "mu")}.get(self.optimizer, ())):
            v = state.get(name)
            if v is None:
                if step:
                    raise KeyError(f"optimizer state at step {step} lacks {name!r}")
                continue
            if isinstance(v, dict):  # torch's per-parameter scalar tensors (all equal)
                v = next(iter(v.values()))
            self._carry[i] = float(v)
        self.step_count = step
        self.first_step = step == 0

    def get_global_model_params(self) -> "OrderedDict[str, torch.Tensor]":
        """Views of the persistent global vectors (built once; they track every
        later aggregate())."""
        if self._views is not None:
            return self._views
        out = OrderedDict()
        for key, shape, _ in self.bucket.entries:
            g, j = self.bucket.where[key]
            if key in self._int_state:
                out[key] = self._int_state[key]
            else:
                out[key] = self.global_flat[g.dtype][g.offsets[j]:g.offsets[j] + g.numels[j]].view(g.shapes[j])
        self._views = out
        return out

    def algorithmic_bytes(self) -> int:
        """Per aggregate(): K rows read once; param runs read p_old (+ mom) and
        write p_new (+ mom); buffer runs write the average."""
        K = self.worker_num
        tot = 0
        for is_param, lo, hi in self.runs:
            n = hi - lo
            tot += K * n * 4
            if not is_param:
                tot += n * 4
            elif self.optimizer in ("adam", "adamw"):  # p read+write, exp_avg / exp_avg_sq written (+ read after step 1)
                tot += 2 * n * 4 + (4 if not self.first_step else 2) * n * 4
            elif self.optimizer in ("adagrad", "rmsprop"):  # p and state_sum / square_avg read and written
                tot += 4 * n * 4
            elif self.optimizer in OPTREPO_STATE:  # p and each state buffer read and written (ASGD: ax written)
                tot += 2 * n * 4 + (2 * len(OPTREPO_STATE[self.optimizer]) * n * 4 if self.optimizer != "asgd"
                                    else n * 4)
            else:
                tot += 2 * n * 4 + (2 * n * 4 if self.mom is not None and not self.first_step else
                                    (n * 4 if self.mom is not None else 0))
        return tot


class MultiDeviceFedOptServer:
    """FedOptServer over G GPUs of ONE server process (the reference's
    FedOptAggregator is one process: FedOptAggregator.py:81-130).

    The model's keys are dealt to the devices whole (multidev.shard_plan, the
    partition MultiDeviceBucket uses) and every device runs an ordinary
    FedOptServer over its keys: its own client rows, global vector and
    optimizer state, its own fused FedAvg + server-step launches.  Every
    element's FedAvg chain and optimizer step are the one-device ones, so the
    result is bit-exact with FedOptServer, and nothing is exchanged.

    It offers FedOptServer's round interface (add_local_trained_result,
    check_whether_all_receive, aggregate, get_global_model_params,
    optimizer_state / load_optimizer_state, sample_num_dict, step_count) and
    its scalar settings (optimizer, lr, momentum, ...).  Where FedOptServer
    has ONE bucket and device, this has one per shard: ``buckets`` and
    ``devices`` (``device`` / ``bucket`` name the first shard's, for code that
    only needs a device to allocate on).  Built by ``make_fedopt_server`` when
    ``args.fedagg_devices`` lists several GPUs or the round does not fit one."""

    def __init__(self, global_state: "OrderedDict[str, torch.Tensor]", param_names: Sequence[str],
                 worker_num: int, server_optimizer: str = "sgd", server_lr: float = 1.0,
                 server_momentum: float = 0.0, devices: Sequence = (), server_weight_decay: Optional[float] = None):
        from .multidev import shard_plan

        devices = [torch.device(d) for d in devices]
        if not devices:
            raise ValueError("MultiDeviceFedOptServer needs at least one device")
        self.entries = [(k, tuple(t.shape), t.dtype) for k, t in global_state.items()]
        plan = shard_plan(self.entries, len(devices))
        self.devices = devices[:len(plan)]
        self.servers: List[FedOptServer] = []
        for sub, dev in zip(plan, self.devices):
            keys = [k for k, _, _ in sub]
            mine = set(keys)
            self.servers.append(FedOptServer(OrderedDict((k, global_state[k]) for k in keys),
                                             [k for k in param_names if k in mine], worker_num,
                                             server_optimizer, server_lr, server_momentum, dev, server_weight_decay))
        self.owner = {k: i for i, s in enumerate(self.servers) for k, _, _ in s.bucket.entries}
        self.worker_num = worker_num
        first = self.servers[0]
        self.optimizer = first.optimizer
        for a in ("lr", "momentum", "betas", "eps", "alpha", "weight_decay", "lr_decay"):
            setattr(self, a, getattr(first, a))
        self.buckets = [s.bucket for s in self.servers]
        self.bucket, self.device = first.bucket, first.device
        self.param_names = list(param_names)
        self.sample_num_dict = _SharedDict(self.servers, "sample_num_dict")
        self.flag_client_model_uploaded_dict = {i: False for i in range(worker_num)}
        self._views: Optional["OrderedDict[str, torch.Tensor]"] = None

    def add_local_trained_result(self, index: int, model_params, sample_num) -> None:
        """:68-72: every device takes its keys of the update; the host keys of
        all devices are packed in one native gather, then the G H2Ds go out
        back to back (MultiDeviceBucket.put's ingest)."""
        from .bucket import gather_jobs

        jobs = [(s, s.bucket.put_prepare(index, model_params, sample_num)) for s in self.servers]
        gather_jobs([j for _, js in jobs for j in js])
        for s, js in jobs:
            s.bucket.put_issue(js)
            s.note_dict(index, model_params)
            s.sample_num_dict[index] = sample_num
            s.flag_client_model_uploaded_dict[index] = True
        dict.__setitem__(self.sample_num_dict, index, sample_num)
        self.flag_client_model_uploaded_dict[index] = True

    def check_whether_all_receive(self) -> bool:
        for idx in range(self.worker_num):
            if not self.flag_client_model_uploaded_dict[idx]:
                return False
        for idx in range(self.worker_num):
            self.flag_client_model_uploaded_dict[idx] = False
        for s in self.servers:
            for idx in range(self.worker_num):
                s.flag_client_model_uploaded_dict[idx] = False
        return True

    def aggregate(self, events=None, device_events=None) -> "OrderedDict[str, torch.Tensor]":
        """Every device's launches are enqueued on its own current stream
        (events, if given, around the first device's fp32 launches;
        device_events[i] around device i's).  The fused launches of ALL
        devices go out in ONE native call (fedagg_wsum_fedopt_batch), so the
        last device starts one launch after the one before it, not one
        Python round of FedOptServer.aggregate later."""
        first = self.servers[0]
        if any(s._aliases_of_client0() for s in self.servers):  # the aliased round: shard by shard
            for i, s in enumerate(self.servers):
                ev = device_events[i] if device_events is not None else (events if i == 0 else None)
                s.aggregate(events=ev)
            return self.get_global_model_params()
        ns = [first.sample_num_dict[i] for i in range(self.worker_num)]
        weights = first.bucket.weights(ns)
        tab, offs = self._combined_table()
        for s, off in zip(self.servers, offs):
            s._refs, s._same = {}, set()
            s.bucket.sync_ingest()
            s._fill(tab, off, kn.weights_for(weights, torch.float32, s.device))
        evs = device_events if device_events is not None else ([events] + [None] * (len(self.servers) - 1)
                                                                if events is not None else None)
        if evs is not None:
            for s, ev in zip(self.servers, evs):
                if ev is not None:
                    ev[0].record(torch.cuda.current_stream(s.device))
        if len(tab):
            nat.check(nat.lib().fedagg_wsum_fedopt_batch(tab, len(tab)), f"fedopt {self.optimizer} launches")
        if evs is not None:
            for s, ev in zip(self.servers, evs):
                if ev is not None:
                    ev[1].record(torch.cuda.current_stream(s.device))
        for s in self.servers:
            if s._int_state or any(dt != torch.float32 and g.length for dt, g in s.bucket.groups.items()):
                with torch.cuda.device(s.device):
                    s._after(weights, self.worker_num)
            else:
                s._after(weights, self.worker_num)
        return self.get_global_model_params()

    def _combined_table(self):
        """Every device's launch descriptors in one array (built once), and
        each device's first index in it."""
        if getattr(self, "_comb", None) is None:
            tabs = [s._table() for s in self.servers]
            offs, n = [], 0
            for t in tabs:
                offs.append(n)
                n += len(t)
            comb = (nat.FedOptLaunch * n)()
            for t, off in zip(tabs, offs):
                if len(t):
                    ctypes.memmove(ctypes.addressof(comb) + off * ctypes.sizeof(nat.FedOptLaunch),
                                   ctypes.addressof(t), ctypes.sizeof(t))
            self._comb = (comb, offs)
        return self._comb

    def get_global_model_params(self) -> "OrderedDict[str, torch.Tensor]":
        if self._views is None:
            parts = [s.get_global_model_params() for s in self.servers]
            self._views = OrderedDict((k, parts[self.owner[k]][k]) for k, _, _ in self.entries)
        return self._views

    @property
    def step_count(self) -> int:
        return self.servers[0].step_count

    def optimizer_state(self) -> Dict[str, object]:
        out: Dict[str, object] = {"step": self.step_count}
        for s in self.servers:
            for name, v in s.optimizer_state().items():
                if isinstance(v, dict):
                    out.setdefault(name, OrderedDict()).update(v)
                elif name != "step":  # a scalar state, the same on every device
                    out[name] = v
        for name, v in list(out.items()):  # the model's parameter order
            if isinstance(v, dict):
                out[name] = OrderedDict((k, v[k]) for k in self.param_names if k in v)
        return out

    def load_optimizer_state(self, state: Dict[str, object]) -> None:
        for s in self.servers:
            mine = {k for k, _, _ in s.bucket.entries}
            s.load_optimizer_state({name: (OrderedDict((k, t) for k, t in v.items() if k in mine)
                                           if isinstance(v, dict) else v)
                                    for name, v in state.items()})

    def algorithmic_bytes(self) -> int:
        return sum(s.algorithmic_bytes() for s in self.servers)


class _SharedDict(dict):
    """sample_num_dict of a MultiDeviceFedOptServer: a write goes to every
    device's server too (the reference sets it per client before aggregate)."""

    def __init__(self, servers, attr):
        super().__init__()
        self._targets = [getattr(s, attr) for s in servers]

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        for t in self._targets:
            t[k] = v


def make_fedopt_server(global_state: "OrderedDict[str, torch.Tensor]", param_names: Sequence[str], worker_num: int,
                       server_optimizer: str = "sgd", server_lr: float = 1.0, server_momentum: float = 0.0,
                       device=None, args=None, server_weight_decay: Optional[float] = None):
    """The FedOpt server for this round's shape: one device, or several GPUs
    of this process when ``args.fedagg_devices`` lists them or the round does
    not fit the default device's free HBM (multidev.devices_for_round, the
    rule FedMLAggOperator.agg and the cross-silo mirror use)."""
    from .multidev import devices_for_round

    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    entries = [(k, tuple(t.shape), t.dtype) for k, t in global_state.items()]
    # the server also holds the global vector and the optimizer state: up to
    # three more model-sized fp32 vectors besides the K + 1 rows
    devs = devices_for_round(args, entries, worker_num + 3, dev)
    if len(devs) > 1:
        return MultiDeviceFedOptServer(global_state, param_names, worker_num, server_optimizer, server_lr,
                                       server_momentum, devs, server_weight_decay)
    return FedOptServer(global_state, param_names, worker_num, server_optimizer, server_lr, server_momentum,
                        devs[0], server_weight_decay)
