"""The server-aggregator plugin surface, with the MI355X reduction behind it.

Mirrors python/fedml/core/alg_frame/server_aggregator.py:14-141 (the
``ServerAggregator`` ABC every FedML server calls: on_before_aggregation ->
aggregate -> on_after_aggregation) and the default subclass of
python/fedml/ml/aggregator/default_aggregator.py:12-23.

``aggregate`` routes to fedml_amd.agg_operator.FedMLAggOperator.agg, the GPU
implementation of the reference's operator.  Two of FedML's defenses are
reductions over the client axis and run on the GPU too (fedml_amd.defense):
``defense_type`` "wise_median" (on aggregation) and "trimmed_mean" (before
aggregation), dispatched exactly as FedMLDefender does
(core/security/fedml_defender.py:131-171).  The other optional hooks (FHE,
differential privacy, attacks, other defenses, contribution assessment) are
outside this build's scope: disabled (FedML's default) they are the identity,
as in the reference; enabling one raises NotImplementedError instead of
silently aggregating without it.

INTEGRATION.md shows the two-line subclass a FedML maintainer adds to route
FedML's own ServerAggregator through this operator.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from collections import OrderedDict
from typing import List, Tuple

from . import defense as dfn
from .agg_operator import FedMLAggOperator

_UNSUPPORTED_FLAGS = ("enable_fhe", "enable_dp", "enable_attack", "enable_contribution")


def _check_flags(args) -> None:
    for flag in _UNSUPPORTED_FLAGS:
        if getattr(args, flag, False):
            raise NotImplementedError(
                f"args.{flag} is set: FedML's {flag[7:]} hooks are not part of fedml_amd; "
                "use FedML's own ServerAggregator for that round")
    if getattr(args, "enable_defense", False):
        dt = str(getattr(args, "defense_type", "")).strip()
        if dt not in dfn.SUPPORTED:
            raise NotImplementedError(f"defense_type {dt!r}: fedml_amd runs {dfn.SUPPORTED} on the GPU")


def _defense(args):
    if not getattr(args, "enable_defense", False):
        return None
    return str(args.defense_type).strip()


class ServerAggregator(ABC):
    """Same interface as fedml.core.alg_frame.server_aggregator.ServerAggregator."""

    def __init__(self, model, args):
        self.model = model
        self.id = 0
        self.args = args
        _check_flags(args)
        self.final_contribution_assigment_dict = dict()
        self.eval_data = None

    def is_main_process(self):
        return True

    def set_id(self, aggregator_id):
        self.id = aggregator_id

    @abstractmethod
    def get_model_params(self):
        pass

    @abstractmethod
    def set_model_params(self, model_parameters):
        pass

    def on_before_aggregation(self, raw_client_model_or_grad_list: List[Tuple[float, OrderedDict]]):
        """server_aggregator.py:44-73 (FHE/DP/attacks disabled); the trimmed-mean
        defense filters the list here (fedml_defender.py:134-161)."""
        client_idxs = [i for i in range(len(raw_client_model_or_grad_list))]
        if _defense(self.args) == dfn.DEFENSE_TRIMMED_MEAN:
            raw_client_model_or_grad_list = dfn.trimmed_mean_before_aggregation(
                raw_client_model_or_grad_list, self.args.beta)
        return raw_client_model_or_grad_list, client_idxs  # no client is flagged malicious

    def aggregate(self, raw_client_model_or_grad_list: List[Tuple[float, OrderedDict]]):
        """server_aggregator.py:75-88: the median defense replaces the operator
        (fedml_defender.py:163-174), otherwise FedMLAggOperator.agg."""
        if _defense(self.args) == dfn.DEFENSE_WISE_MEDIAN:
            return dfn.coordinate_wise_median(raw_client_model_or_grad_list, getattr(self.args, "fedagg_device", None))
        return FedMLAggOperator.agg(self.args, raw_client_model_or_grad_list)

    def on_after_aggregation(self, aggregated_model_or_grad: OrderedDict) -> OrderedDict:
        """server_aggregator.py:90-103 with DP/defense disabled."""
        return aggregated_model_or_grad

    def assess_contribution(self):
        return None

    @abstractmethod
    def test(self, test_data, device, args):
        pass

    def test_all(self, train_data_local_dict, test_data_local_dict, device, args) -> bool:
        pass


class MI355XServerAggregator(ServerAggregator):
    """DefaultServerAggregator (default_aggregator.py:12-23) on MI355X:
    state_dict in, load_state_dict out, FedAvg on the GPU."""

    def __init__(self, model, args):
        super().__init__(model, args)
        self.cpu_transfer = False if not hasattr(self.args, "cpu_transfer") else self.args.cpu_transfer

    def get_model_params(self):
        if self.cpu_transfer:
            return self.model.cpu().state_dict()
        return self.model.state_dict()

    def set_model_params(self, model_parameters):
        self.model.load_state_dict(model_parameters)

    def test(self, test_data, device, args):
        return None


class _TaskEvalServerAggregator(MI355XServerAggregator):
    """MyServerAggregatorNWP / MyServerAggregatorTAGPred
    (my_server_aggregator_nwp.py:12-50, my_server_aggregator_prediction.py:12-67):
    the same state-dict exchange and aggregation as the default aggregator;
    they differ only in task-specific evaluation, which is outside the
    aggregation path and raises here instead of reporting
    nothing."""

    def get_model_params(self):
        return self.model.cpu().state_dict()  # :13-14 of both: always the host copy

    def test(self, test_data, device, args):
        raise NotImplementedError(f"server-side evaluation for dataset {getattr(args, 'dataset', None)!r} "
                                  "is out of scope (fedml_amd rebuilds the aggregation path)")


def create_server_aggregator(model, args) -> ServerAggregator:
    """aggregator_creator.py:6-13: the dataset picks the class; every one of
    them aggregates through FedMLAggOperator.agg on the GPU here."""
    if getattr(args, "dataset", None) in ("stackoverflow_lr", "fed_shakespeare", "stackoverflow_nwp"):
        return _TaskEvalServerAggregator(model, args)
    return MI355XServerAggregator(model, args)
