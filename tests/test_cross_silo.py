"""Host logic of the cross-silo FedMLAggregator mirror (no GPU): arrival
bookkeeping, the CPU-server move, and the seeded client draws of
fedml_aggregator.py:113-165."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from fedml_amd.cross_silo import FedMLAggregator


class _Args:
    federated_optimizer = "FedAvg"


def _server(K, device="cpu"):
    return FedMLAggregator(None, None, 0, {}, {}, {}, K, torch.device(device), _Args(), None)


def test_arrival_bookkeeping_on_a_cpu_server():
    """device = cpu: no bucket (it lives in HBM); updates are moved key by key
    as model_params_to_device does, and check_whether_all_receive resets the
    flags once every client has arrived (:69-76)."""
    s = _server(2)
    d = OrderedDict(w=torch.ones(3))
    s.add_local_trained_result(0, d, 10)
    assert not s.check_whether_all_receive()
    s.add_local_trained_result(1, OrderedDict(w=torch.zeros(3)), 30)
    assert s.bucket is None and s.model_dict[0] is d and s.sample_num_dict == {0: 10, 1: 30}
    assert s.check_whether_all_receive()
    assert not s.check_whether_all_receive()
    assert s.args.device == torch.device("cpu")


def test_client_draws_match_the_reference_numpy_calls():
    s = _server(4)
    np.random.seed(7)
    exp = np.random.choice(range(30), 5, replace=False)
    assert list(s.client_sampling(7, 30, 5)) == list(exp)
    assert s.client_sampling(1, 5, 5) == [0, 1, 2, 3, 4]
    assert s.data_silo_selection(0, 3, 3) == [0, 1, 2]
    np.random.seed(4)
    exp = np.random.choice(range(9), 3, replace=False)
    assert list(s.data_silo_selection(4, 9, 3)) == list(exp)
    np.random.seed(2)
    exp = np.random.choice([64, 65, 66, 67], 2, replace=False)
    assert list(s.client_selection(2, [64, 65, 66, 67], 2)) == list(exp)
    assert s.client_selection(2, [64, 65], 2) == [64, 65]


def test_create_server_aggregator_picks_by_dataset():
    """aggregator_creator.py:6-13: task-specific classes only change evaluation."""
    from fedml_amd.server_aggregator import MI355XServerAggregator, create_server_aggregator

    class A:
        dataset = "mnist"

    agg = create_server_aggregator(torch.nn.Linear(2, 2), A())
    assert type(agg) is MI355XServerAggregator and agg.test(None, None, A()) is None
    A.dataset = "stackoverflow_nwp"
    agg = create_server_aggregator(torch.nn.Linear(2, 2), A())
    assert isinstance(agg, MI355XServerAggregator)
    try:
        agg.test(None, None, A())
        raise AssertionError("task evaluation should raise")
    except NotImplementedError:
        pass
