"""The single-process simulators' copy of the FedAvg reduction, on MI355X.

FedAvgAPI._aggregate (python/fedml/simulation/sp/fedavg/fedavg_api.py:144-159)
and FedOptAPI._aggregate (sp/fedopt/fedopt_api.py:143-158) restate the plugin
operator's FedAvg loop without ``args``: Σn with a Python loop, then
avg[k] = p_0[k]·w_0, avg[k] += p_i[k]·w_i, w_i = n_i / Σn, rebinding the keys of
client 0's dict.  ``fedavg_aggregate`` keeps that contract (same unpacking and
so the same ValueError, ZeroDivisionError at Σn = 0, the same returned object)
and runs the reduction in libfedagg.so through fedml_amd.agg_operator.

A simulator swaps the method in one line:

    FedAvgAPI._aggregate = lambda self, w_locals: fedavg_aggregate(w_locals)

The MPI simulator's FedAVGAggregator._fedavg_aggregation_
(simulation/mpi/fedavg/FedAVGAggregator.py:99-116) writes each term as
``local_model_params[k] * local_sample_number / training_num``: two roundings
per client, fl(fl(p·n_i)/N), in a different order from the plugin path's
fl(p·fl(n_i/N)).  ``fedavg_mpi_aggregate`` reproduces that order bit for bit
(fedagg_wsum_muldiv):

    FedAVGAggregator._fedavg_aggregation_ = lambda self, model_list: fedavg_mpi_aggregate(model_list)
"""
from __future__ import annotations

from typing import List, Tuple

from .agg_operator import _reads_running_cell, _run_cells, muldiv_reduce, weighted_reduce


class _Defaults:
    """The reduction options fedml_amd reads from FedML's args, at their defaults."""

    fedagg_low_precision_acc = "reference"
    fedagg_device = None


def fedavg_aggregate(w_locals: List[Tuple[float, "OrderedDict"]], args=None) -> "OrderedDict":
    """fedavg_api.py:144-159.  ``args`` (optional) may carry the fedml_amd
    options ``fedagg_device`` / ``fedagg_low_precision_acc``.  Client 0's
    dict listed again reads the running average, as the reference's
    rebind-then-``+=`` loop makes it (fedml_amd.agg_operator._run_cells, the
    rule torch_aggregator follows)."""
    training_num = 0
    for idx in range(len(w_locals)):
        (sample_num, averaged_params) = w_locals[idx]
        training_num += sample_num
    (sample_num, averaged_params) = w_locals[0]
    keys = list(averaged_params.keys())
    if not keys:
        return averaged_params
    weights = [w_locals[i][0] / training_num for i in range(len(w_locals))]
    a = args if args is not None else _Defaults()
    if _reads_running_cell(w_locals, (1,)):  # client 0's dict listed again reads the running sum (:150-158)
        _run_cells(w_locals, (1,), keys, weights, a)
        return averaged_params
    res = weighted_reduce([w_locals[i][1] for i in range(len(w_locals))], keys, weights, a)
    for k in keys:
        averaged_params[k] = res[k]
    return averaged_params


def fedavg_mpi_aggregate(model_list: List[Tuple[float, "OrderedDict"]], args=None) -> "OrderedDict":
    """FedAVGAggregator._fedavg_aggregation_ (FedAVGAggregator.py:99-116): the
    same unpacking, Σn loop and returned object (client 0's dict, keys
    rebound), each term fl(fl(p·n_i)/Σn).  Σn = 0 divides tensors by zero as
    torch does (inf / NaN, no exception).  Client 0's dict listed again reads
    the running sum, as in the reference (fedml_amd.agg_operator._run_cells)."""
    training_num = 0
    for i in range(0, len(model_list)):
        local_sample_number, local_model_params = model_list[i]
        training_num += local_sample_number
    (num0, averaged_params) = model_list[0]
    keys = list(averaged_params.keys())
    if not keys:
        return averaged_params
    a = args if args is not None else _Defaults()
    pairs = [(model_list[i][0], training_num) for i in range(len(model_list))]
    if _reads_running_cell(model_list, (1,)):
        _run_cells(model_list, (1,), keys, pairs, a, reduce=muldiv_reduce, one=(1, 1))
        return averaged_params
    res = muldiv_reduce([model_list[i][1] for i in range(len(model_list))], keys, pairs, a)
    for k in keys:
        averaged_params[k] = res[k]
    return averaged_params
