"""The server-aggregator plugin surface, with the MI355X reduction behind it.

Mirrors python/fedml/core/alg_frame/server_aggregator.py:14-141 (the
``ServerAggregator`` ABC every FedML server calls: on_before_aggregation ->
aggregate -> on_after_aggregation) and the default subclass of
python/fedml/ml/aggregator/default_aggregator.py:12-23.

``aggregate`` routes to fedml_amd.agg_operator.FedMLAggOperator.agg, the GPU
implementation of the reference's operator.  Several of FedML's defenses are
reductions over the client axis and run on the GPU too (fedml_amd.defense):
``defense_type`` "wise_median" (on aggregation) and "trimmed_mean" (before
aggregation), dispatched exactly as FedMLDefender does
(core/security/fedml_defender.py:131-171); so do the distance-based
"krum" / "multikrum", "norm_diff_clipping", "slsgd" and "cclip".  "robust_learning_rate" and
"weak_dp" are accepted and, as in FedML, leave the plugin path a plain FedAvg
(FedMLDefender lists them under none of the three hooks; the GPU version of the
first, fedml_amd.defense.RobustLearningRateDefense, runs where FedML calls
FedMLDefender.defend).  The other optional hooks (FHE,
differential privacy, attacks, other defenses, contribution assessment) are
outside this build's scope: disabled (FedML's default) they are the identity,
as in the reference; enabling one raises NotImplementedError instead of
silently aggregating without it.

INTEGRATION.md shows the two-line subclass a FedML maintainer adds to route
FedML's own ServerAggregator through this operator.
"""
from __future__ import annotations

import copy
import logging
from abc import ABC, abstractmethod
from collections import OrderedDict
from typing import List, Tuple

import torch
from torch import nn

from . import defense as dfn
from .agg_operator import FedMLAggOperator

_UNSUPPORTED_FLAGS = ("enable_fhe", "enable_dp", "enable_attack", "enable_contribution")


# attributes each defender's __init__ reads (krum_defense.py, norm_diff_clipping_
# defense.py, cclip_defense.py, slsgd_defense.py; FedMLDefender.init builds it)
_DEFENSE_ATTRS = {
    dfn.DEFENSE_KRUM: ("byzantine_client_num",),
    dfn.DEFENSE_MULTIKRUM: ("byzantine_client_num",),
    dfn.DEFENSE_NORM_DIFF_CLIPPING: ("norm_bound",),
    dfn.DEFENSE_CCLIP: ("bucket_size",),
    dfn.DEFENSE_SLSGD: ("trim_param_b",),  # then the alpha check, then option_type
}


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
        # the defender's constructor reads these at FedMLDefender.init, so a
        # missing one fails at construction there, not at the first round
        for attr in _DEFENSE_ATTRS.get(dt, ()):
            getattr(args, attr)
        if dt == dfn.DEFENSE_SLSGD:
            dfn.slsgd_alpha_check(args.alpha)  # SLSGDDefense.__init__ raises at FedMLDefender.init
            args.option_type
        if dt == dfn.DEFENSE_ROBUST_LEARNING_RATE:
            args.robust_threshold  # RobustLearningRateDefense.__init__ reads it at FedMLDefender.init
        if dt == dfn.DEFENSE_WEAK_DP:
            args.stddev  # WeakDPDefense.__init__ (weak_dp_defense.py:12-14)


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
        self._cclip_guess = None  # CClip's initial guess, kept from before to after aggregation

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
        """server_aggregator.py:44-73 (FHE/DP/attacks disabled); the
        before-aggregation defenses (trimmed mean, Krum / multi-Krum, norm-diff
        clipping) rewrite the list here (fedml_defender.py:134-161)."""
        client_idxs = [i for i in range(len(raw_client_model_or_grad_list))]
        dt = _defense(self.args)
        dev = getattr(self.args, "fedagg_device", None)
        if dt == dfn.DEFENSE_TRIMMED_MEAN:
            raw_client_model_or_grad_list = dfn.trimmed_mean_before_aggregation(
                raw_client_model_or_grad_list, self.args.beta)
        elif dt in (dfn.DEFENSE_KRUM, dfn.DEFENSE_MULTIKRUM):
            raw_client_model_or_grad_list = dfn.krum_before_aggregation(
                raw_client_model_or_grad_list, self.args.byzantine_client_num, dfn.krum_param_m(self.args), dev,
                getattr(self.args, "fedagg_pair_distance", "auto"))
        elif dt == dfn.DEFENSE_NORM_DIFF_CLIPPING:
            # extra_auxiliary_info = the server's current model (server_aggregator.py:66-70)
            raw_client_model_or_grad_list = dfn.norm_diff_clipping_before_aggregation(
                raw_client_model_or_grad_list, self.get_model_params(), self.args.norm_bound, dev)
        elif dt == dfn.DEFENSE_SLSGD:
            raw_client_model_or_grad_list = dfn.slsgd_before_aggregation(
                raw_client_model_or_grad_list, self.args.trim_param_b, self.args.option_type)
        elif dt == dfn.DEFENSE_CCLIP:
            raw_client_model_or_grad_list, self._cclip_guess = dfn.cclip_before_aggregation(
                raw_client_model_or_grad_list, dfn.cclip_tau(self.args), self.args.bucket_size, dev)
        return raw_client_model_or_grad_list, client_idxs  # no client is flagged malicious

    def aggregate(self, raw_client_model_or_grad_list: List[Tuple[float, OrderedDict]]):
        """server_aggregator.py:75-88: the median defense replaces the operator
        (fedml_defender.py:163-174), otherwise FedMLAggOperator.agg."""
        if _defense(self.args) == dfn.DEFENSE_WISE_MEDIAN:
            return dfn.coordinate_wise_median(raw_client_model_or_grad_list, getattr(self.args, "fedagg_device", None))
        if _defense(self.args) == dfn.DEFENSE_SLSGD:
            # defend_on_aggregation (slsgd_defense.py:54-67): the base operator, then the
            # moving average with the global model (extra_auxiliary_info, :81-85)
            avg = FedMLAggOperator.agg(self.args, raw_client_model_or_grad_list)
            return dfn.slsgd_on_aggregation(avg, self.get_model_params(), self.args.alpha,
                                            getattr(self.args, "fedagg_device", None))
        return FedMLAggOperator.agg(self.args, raw_client_model_or_grad_list)

    def on_after_aggregation(self, aggregated_model_or_grad: OrderedDict) -> OrderedDict:
        """server_aggregator.py:90-103 with DP disabled: CClip adds its
        initial guess back (fedml_defender.py:149-150, cclip_defense.py:57-60);
        the other defenses pass the model through."""
        if _defense(self.args) == dfn.DEFENSE_CCLIP:
            return dfn.cclip_after_aggregation(aggregated_model_or_grad, self._cclip_guess,
                                               getattr(self.args, "fedagg_device", None))
        return aggregated_model_or_grad

    def assess_contribution(self):
        return None

    @abstractmethod
    def test(self, test_data, device, args):
        pass

    def test_all(self, train_data_local_dict, test_data_local_dict, device, args) -> bool:
        pass


def _evaluate(model, test_data, device, task: str) -> dict:
    """The `_test` loops of default_aggregator.py:25-75 ("classification", and
    its stackoverflow_lr branch "default_multilabel": BCE and the precision /
    recall sums, with the default class's test_total rule, size(0) for 1-D
    targets and size(0)*size(1) for 2-D ones, :71-74), my_server_aggregator_
    prediction.py:19-60 ("tag_prediction": test_total += size(0)) and
    my_server_aggregator_nwp.py:19-43 ("nwp"): the same criteria, predictions
    and metric sums.  Server
    evaluation is model inference, not aggregation; it runs with torch on
    `device` exactly as in the reference."""
    model.to(device)
    model.eval()
    metrics = {"test_correct": 0, "test_loss": 0, "test_total": 0}
    multilabel = task in ("tag_prediction", "default_multilabel")
    if multilabel:
        metrics.update(test_precision=0, test_recall=0)
        criterion = nn.BCELoss(reduction="sum").to(device)
    elif task == "nwp":
        criterion = nn.CrossEntropyLoss(ignore_index=0).to(device)
    else:
        metrics.update(test_precision=0, test_recall=0)
        criterion = nn.CrossEntropyLoss().to(device)
    with torch.no_grad():
        for batch_idx, (x, target) in enumerate(test_data):
            x = x.to(device)
            target = target.to(device)
            pred = model(x)
            loss = criterion(pred, target)
            if multilabel:
                predicted = (pred > 0.5).int()
                correct = predicted.eq(target).sum(axis=-1).eq(target.size(1)).sum()
                true_positive = ((target * predicted) > 0.1).int().sum(axis=-1)
                metrics["test_precision"] += (true_positive / (predicted.sum(axis=-1) + 1e-13)).sum().item()
                metrics["test_recall"] += (true_positive / (target.sum(axis=-1) + 1e-13)).sum().item()
            elif task == "nwp":
                _, predicted = torch.max(pred, 1)
                target_pos = ~(target == 0)
                correct = (predicted.eq(target) * target_pos).sum()
            else:
                _, predicted = torch.max(pred, 1)
                correct = predicted.eq(target).sum()
            metrics["test_correct"] += correct.item()
            metrics["test_loss"] += loss.item() * target.size(0)
            if task == "nwp":
                metrics["test_total"] += target_pos.sum().item()
            elif task == "tag_prediction" or len(target.size()) == 1:
                metrics["test_total"] += target.size(0)
            elif len(target.size()) == 2:  # next-word prediction targets through the default class
                metrics["test_total"] += target.size(0) * target.size(1)
    return metrics


def _report(args, round_args, metrics) -> tuple:
    """default_aggregator.py:77-106: accuracy and mean loss over the test
    set, logged, returned as the four-metric tuple the server stores in its
    Context (fedml_aggregator.py:193-202).  mlops is outside this build;
    wandb is logged when enabled, as in the reference."""
    test_tot_corrects = [copy.deepcopy(metrics["test_correct"])]
    test_num_samples = [copy.deepcopy(metrics["test_total"])]
    test_losses = [copy.deepcopy(metrics["test_loss"])]
    test_acc = sum(test_tot_corrects) / sum(test_num_samples)
    test_loss = sum(test_losses) / sum(test_num_samples)
    if getattr(args, "enable_wandb", False):
        import wandb  # the reference imports it unconditionally

        wandb.log({"Test/Acc": test_acc, "round": round_args.round_idx})
        wandb.log({"Test/Loss": test_loss, "round": round_args.round_idx})
    logging.info({"test_acc": test_acc, "test_loss": test_loss})
    return (test_acc, test_loss, None, None)


def _plain_load(model) -> bool:
    """load_state_dict would do nothing to this model's values but copy_ them:
    no load-state-dict pre / post hooks on any submodule (nor the model-level
    ones), and no _load_from_state_dict override besides torch's BatchNorm one
    (_NormBase's only fills in a missing num_batches_tracked of an old
    checkpoint; the fast path passes every key)."""
    from torch.nn.modules.batchnorm import _NormBase

    for m in model.modules():
        if getattr(m, "_load_state_dict_pre_hooks", None) or getattr(m, "_load_state_dict_post_hooks", None):
            return False
        f = type(m)._load_from_state_dict
        if f is not torch.nn.Module._load_from_state_dict and f is not _NormBase._load_from_state_dict:
            return False
    return True


class MI355XServerAggregator(ServerAggregator):
    """DefaultServerAggregator (default_aggregator.py:12-106) on MI355X:
    state_dict in, load_state_dict out, FedAvg on the GPU, and the
    reference's server-side evaluation in test()."""

    _task = "classification"

    def __init__(self, model, args):
        super().__init__(model, args)
        self.cpu_transfer = False if not hasattr(self.args, "cpu_transfer") else self.args.cpu_transfer

    def get_model_params(self):
        if self.cpu_transfer:
            return self.model.cpu().state_dict()
        return self.model.state_dict()

    def set_model_params(self, model_parameters):
        """load_state_dict (default_aggregator.py:25-27).  When the server
        model lives in host memory and the averaged tensors on the GPU, the
        copy goes buffer by buffer (fedml_amd.host_copy: one DMA per flat
        result buffer straight into the model's tensors) instead of one
        pageable D2H per key; the key set must be the model's, as with
        load_state_dict's strict check."""
        sd = self.model.state_dict()
        if (isinstance(model_parameters, dict) and list(sd) == list(model_parameters)
                and all(not t.is_cuda for t in sd.values())
                and any(isinstance(t, torch.Tensor) and t.is_cuda for t in model_parameters.values())):
            from .host_copy import to_host

            if not _plain_load(self.model):
                # a module transforms values on load (its own _load_from_state_dict
                # or load hooks): load_state_dict runs them, on host tensors
                # copied one DMA per result buffer instead of one D2H per key
                self.model.load_state_dict(to_host(model_parameters))
                return
            host = to_host(model_parameters, into=sd)
            # keys written in place are the model's own tensors, so bump their
            # version counters as load_state_dict's copy_ does; the rest
            # (another dtype, e.g. int64 counters from float32 averages) take
            # load_state_dict's conversion
            for k, v in host.items():
                if v is sd[k]:
                    torch.autograd.graph.increment_version(v)
            rest = OrderedDict((k, v) for k, v in host.items() if v is not sd[k])
            if rest:
                self.model.load_state_dict(rest, strict=False)
            return
        self.model.load_state_dict(model_parameters)

    def _test(self, test_data, device, args):
        task = self._task
        if task == "classification" and getattr(args, "dataset", None) == "stackoverflow_lr":
            task = "default_multilabel"  # default_aggregator.py:45-63
        return _evaluate(self.model, test_data, device, task)

    def test(self, test_data, device, args):
        """-> (test_acc, test_loss, None, None), default_aggregator.py:77-106."""
        return _report(self.args, args, self._test(test_data, device, args))


class MI355XServerAggregatorTAGPred(MI355XServerAggregator):
    """MyServerAggregatorTAGPred (my_server_aggregator_prediction.py:12-90):
    the host copy of the model, multi-label (BCE) evaluation."""

    _task = "tag_prediction"

    def get_model_params(self):
        return self.model.cpu().state_dict()  # :13-14


class MI355XServerAggregatorNWP(MI355XServerAggregator):
    """MyServerAggregatorNWP (my_server_aggregator_nwp.py:12-72): the host copy
    of the model, next-word-prediction evaluation (padding id 0 ignored)."""

    _task = "nwp"

    def get_model_params(self):
        return self.model.cpu().state_dict()  # :13-14


def create_server_aggregator(model, args) -> ServerAggregator:
    """aggregator_creator.py:6-13: the dataset picks the class; every one of
    them aggregates through FedMLAggOperator.agg on the GPU here."""
    if args.dataset == "stackoverflow_lr":
        return MI355XServerAggregatorTAGPred(model, args)
    if args.dataset in ("fed_shakespeare", "stackoverflow_nwp"):
        return MI355XServerAggregatorNWP(model, args)
    return MI355XServerAggregator(model, args)
