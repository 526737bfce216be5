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

Supported server optimizer: "sgd" (OptRepo name, optrepo.py:10), with or
without momentum — the optimizers the MPI aggregator can build (it passes
`momentum=` to the constructor).  Parameters are fp32.

Device layout: the round's updates sit in a ClientBucket; the global model
and the momentum buffers are flat fp32 vectors with the bucket's fp32 layout.
Every maximal run of consecutive parameter keys is ONE fused launch
(fedagg_wsum_fedopt_sgd_f32: the average never reaches HBM), every run of
buffer keys one plain FedAvg launch writing straight into the global vector.
For a LoRA adapter set (config 5) all keys are parameters: one launch.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import kernels as kn
from .bucket import ClientBucket


class FedOptServer:
    def __init__(self, global_state: "OrderedDict[str, torch.Tensor]", param_names: Sequence[str],
                 worker_num: int, server_optimizer: str = "sgd", server_lr: float = 1.0,
                 server_momentum: float = 0.0, device=None):
        if server_optimizer.lower() != "sgd":
            raise NotImplementedError(f"server_optimizer {server_optimizer!r}: only 'sgd' (with momentum) is fused")
        self.lr = float(server_lr)
        self.momentum = float(server_momentum)
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
        self.first_step = True
        self._views: Optional["OrderedDict[str, torch.Tensor]"] = None
        self.runs: List[Tuple[bool, int, int]] = self._runs(f32) if f32 else []
        self.run_ptrs = [kn.upload_i64([f32.rows[i].data_ptr() + lo * 4 for i in range(worker_num)], self.device)
                         for _, lo, _ in self.runs]
        self.model_dict: Dict[int, "OrderedDict"] = {}
        self.sample_num_dict: Dict[int, float] = {}
        self.flag_client_model_uploaded_dict = {i: False for i in range(worker_num)}

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
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

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
        K = self.worker_num
        with torch.cuda.device(self.device):
            self.bucket.sync_ingest()
            w32 = kn.weights_for(weights, torch.float32, self.device)  # by value for K <= 256
            f32 = self.global_flat.get(torch.float32)
            if events is not None:
                events[0].record()
            for (is_param, lo, hi), d_ptrs in zip(self.runs, self.run_ptrs):
                if is_param:
                    kn.wsum_fedopt_sgd(d_ptrs, w32, K, hi - lo, f32[lo:hi],
                                       self.mom[lo:hi] if self.mom is not None else None,
                                       self.lr, self.momentum, self.first_step, True)
                else:
                    kn.wsum_ptrs(torch.float32, d_ptrs, w32, K, hi - lo, f32[lo:hi], True)
            if events is not None:
                events[1].record()
            for dt, g in self.bucket.groups.items():
                if dt == torch.float32 or g.length == 0:
                    continue
                w = kn.weights_for(weights, dt, self.device)
                kn.wsum_ptrs(dt, g.d_ptrs, w, K, g.length, self.global_flat[dt], True)
            for k, t in self._int_state.items():
                # load_state_dict's copy_: the float32 average truncates toward zero
                g, j = self.bucket.where[k]
                t.reshape(-1).copy_(self.global_flat[g.dtype][g.offsets[j]:g.offsets[j] + g.numels[j]])
        self.first_step = False
        return self.get_global_model_params()

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
            tot += (2 * n * 4 + (2 * n * 4 if self.mom is not None and not self.first_step else
                                 (n * 4 if self.mom is not None else 0))) if is_param else n * 4
        return tot
