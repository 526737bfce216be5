"""The server-aggregator plugin surface, with the MI355X reduction behind it.

Mirrors python/fedml/core/alg_frame/server_aggregator.py:14-141 (the
``ServerAggregator`` ABC every FedML server calls: on_before_aggregation ->
aggregate -> on_after_aggregation) and the default subclass of
python/fedml/ml/aggregator/default_aggregator.py:12-23.

``aggregate`` routes to fedml_amd.agg_operator.FedMLAggOperator.agg, the GPU
implementation of the reference's operator.  The reference's optional hooks
(FHE, differential privacy, attacks, defenses, contribution assessment) are
outside this build's scope: with them disabled (FedML's default) the hooks are
the identity, exactly as in the reference; enabling one raises
NotImplementedError instead of silently aggregating without it.

INTEGRATION.md shows the two-line subclass a FedML maintainer adds to route
FedML's own ServerAggregator through this operator.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from collections import OrderedDict
from typing import List, Tuple

from .agg_operator import FedMLAggOperator

_UNSUPPORTED_FLAGS = ("enable_fhe", "enable_dp", "enable_defense", "enable_attack", "enable_contribution")


def _check_flags(args) -> None:
    for flag in _UNSUPPORTED_FLAGS:
        if getattr(args, flag, False):
            raise NotImplementedError(
                f"args.{flag} is set: FedML's {flag[7:]} hooks are not part of fedml_amd; "
                "use FedML's own ServerAggregator for that round")


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
        """server_aggregator.py:44-73 with FHE/DP/attack/defense disabled."""
        client_idxs = [i for i in range(len(raw_client_model_or_grad_list))]
        return raw_client_model_or_grad_list, client_idxs

    def aggregate(self, raw_client_model_or_grad_list: List[Tuple[float, OrderedDict]]):
        """server_aggregator.py:75-88: FedMLAggOperator.agg(self.args, list)."""
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
