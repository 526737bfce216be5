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

    from fedml_amd.server_aggregator import MI355XServerAggregatorNWP, MI355XServerAggregatorTAGPred

    agg = create_server_aggregator(torch.nn.Linear(2, 2), A())
    assert type(agg) is MI355XServerAggregator
    A.dataset = "stackoverflow_nwp"
    assert type(create_server_aggregator(torch.nn.Linear(2, 2), A())) is MI355XServerAggregatorNWP
    A.dataset = "fed_shakespeare"
    assert type(create_server_aggregator(torch.nn.Linear(2, 2), A())) is MI355XServerAggregatorNWP
    A.dataset = "stackoverflow_lr"
    assert type(create_server_aggregator(torch.nn.Linear(2, 2), A())) is MI355XServerAggregatorTAGPred


class _EvalArgs:
    federated_optimizer = "FedAvg"
    dataset = "mnist"
    round_idx = 0
    enable_wandb = False


def _loader(n=37, d=8, classes=3, seed=0, batch=10):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, d, generator=g)
    y = torch.randint(0, classes, (n,), generator=g)
    return torch.utils.data.DataLoader(torch.utils.data.TensorDataset(x, y), batch_size=batch), x, y


def test_server_test_returns_the_reference_metrics():
    """default_aggregator.py:25-106: test() evaluates the server model and
    returns (acc, loss, None, None): acc = correct / total, loss = the
    batch-mean cross entropy re-weighted by batch size, over the set."""
    from fedml_amd.server_aggregator import MI355XServerAggregator

    torch.manual_seed(1)
    model = torch.nn.Linear(8, 3)
    loader, x, y = _loader()
    res = MI355XServerAggregator(model, _EvalArgs()).test(loader, torch.device("cpu"), _EvalArgs())
    assert isinstance(res, tuple) and len(res) == 4 and res[2] is None and res[3] is None
    with torch.no_grad():
        pred = model(x)
        acc = (pred.argmax(1) == y).sum().item() / len(y)
        loss = sum(torch.nn.functional.cross_entropy(model(x[i:i + 10]), y[i:i + 10]).item() * len(y[i:i + 10])
                   for i in range(0, len(y), 10)) / len(y)
    assert res[0] == acc
    assert abs(res[1] - loss) < 1e-12


def test_server_test_tag_prediction_and_nwp():
    """The multi-label (stackoverflow_lr) and next-word (padding id 0
    ignored) evaluations of my_server_aggregator_prediction.py:19-60 and
    my_server_aggregator_nwp.py:19-43."""
    from fedml_amd.server_aggregator import create_server_aggregator

    class A(_EvalArgs):
        dataset = "stackoverflow_lr"

    torch.manual_seed(2)
    model = torch.nn.Sequential(torch.nn.Linear(6, 4), torch.nn.Sigmoid())
    g = torch.Generator().manual_seed(3)
    x = torch.randn(20, 6, generator=g)
    y = (torch.rand(20, 4, generator=g) > 0.5).float()
    loader = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(x, y), batch_size=7)
    acc, loss, _, _ = create_server_aggregator(model, A()).test(loader, torch.device("cpu"), A())
    with torch.no_grad():
        p = model(x)
        exp_acc = ((p > 0.5).int().eq(y).sum(-1) == 4).sum().item() / 20
        exp_loss = sum(torch.nn.functional.binary_cross_entropy(model(x[i:i + 7]), y[i:i + 7], reduction="sum").item()
                       * len(y[i:i + 7]) for i in range(0, 20, 7)) / 20
    # (the summation order of torch's CPU BCE differs by host ISA: 6.7e-7 apart
    # on a GPU box's host, bit-equal in the build container)
    assert acc == exp_acc and abs(loss - exp_loss) < 1e-5

    A.dataset = "stackoverflow_nwp"
    emb = torch.nn.Sequential(torch.nn.Embedding(11, 5), torch.nn.Flatten(), torch.nn.Linear(15, 11))
    xs = torch.randint(0, 11, (12, 3), generator=g)
    ys = torch.randint(0, 11, (12,), generator=g)
    ys[::3] = 0  # padding targets do not count
    loader = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(xs, ys), batch_size=5)
    acc, loss, _, _ = create_server_aggregator(emb, A()).test(loader, torch.device("cpu"), A())
    with torch.no_grad():
        pred = emb(xs).argmax(1)
        pos = ys != 0
        exp_acc = ((pred == ys) & pos).sum().item() / pos.sum().item()
    assert acc == exp_acc and loss > 0


def test_default_aggregator_counts_2d_targets_on_stackoverflow_lr():
    """DefaultServerAggregator on stackoverflow_lr (default_aggregator.py:45-74)
    uses BCE and the multi-label metrics, but counts test_total as
    size(0) * size(1) for a 2-D target (:71-74); the task-specific
    MyServerAggregatorTAGPred counts size(0) (my_server_aggregator_prediction.py)."""
    from fedml_amd.server_aggregator import MI355XServerAggregator, MI355XServerAggregatorTAGPred

    class A(_EvalArgs):
        dataset = "stackoverflow_lr"

    torch.manual_seed(4)
    model = torch.nn.Sequential(torch.nn.Linear(6, 4), torch.nn.Sigmoid())
    g = torch.Generator().manual_seed(5)
    x = torch.randn(20, 6, generator=g)
    y = (torch.rand(20, 4, generator=g) > 0.5).float()
    loader = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(x, y), batch_size=7)
    d = MI355XServerAggregator(model, A())._test(loader, torch.device("cpu"), A())
    t = MI355XServerAggregatorTAGPred(model, A())._test(loader, torch.device("cpu"), A())
    assert d["test_total"] == 20 * 4 and t["test_total"] == 20
    assert d["test_correct"] == t["test_correct"] and d["test_loss"] == t["test_loss"]
    assert d["test_precision"] == t["test_precision"] and d["test_recall"] == t["test_recall"]


def test_dummy_input_and_shape_type():
    """fedml_aggregator.py:211-258: the first sample of the test loader's
    first batch, all tensors but the label; "int" for integer dtypes."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(9, 3, 4, generator=g)
    tok = torch.randint(0, 5, (9, 7), generator=g)
    y = torch.randint(0, 2, (9,), generator=g)
    loader = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(x, tok, y), batch_size=4)
    s = FedMLAggregator(None, loader, 0, {}, {}, {}, 2, torch.device("cpu"), _Args(), None)
    feats = s.get_dummy_input_tensor()
    assert len(feats) == 2 and torch.equal(feats[0], x[:1]) and torch.equal(feats[1], tok[:1])
    assert s.get_input_shape_type() == ([[1, 3, 4], [1, 7]], ["float", "int"])
    # no server test set: the first non-empty client loader
    s2 = FedMLAggregator(None, None, 0, {}, {0: None, 1: loader}, {}, 2, torch.device("cpu"), _Args(), None)
    assert s2.get_input_shape_type() == ([[1, 3, 4], [1, 7]], ["float", "int"])


def test_rmsprop_server_momentum_is_refused():
    """torch's RMSprop applies `momentum=` and the MPI FedOptAggregator passes
    server_momentum (FedOptAggregator.py:49-54): the fused momentum-free step
    must not stand in for it."""
    import pytest

    from fedml_amd.fedopt import FedOptServer
    from fedml_amd.sharded import ShardedFedOpt

    sd = OrderedDict(w=torch.zeros(4))
    with pytest.raises(NotImplementedError, match="rmsprop"):
        FedOptServer(sd, ["w"], 2, "rmsprop", 0.1, 0.9, "cpu")
    with pytest.raises(NotImplementedError, match="rmsprop"):
        ShardedFedOpt(torch.zeros(2, 4), 4, torch.zeros(4), "rmsprop", 0.1, 0.9, reducer=lambda *a: None)


class _RoundArgs:
    federated_optimizer = "FedAvg"
    dataset = "mnist"
    enable_wandb = False

    def __init__(self, K, comm_round=3, freq=2):
        self.round_idx = 0
        self.comm_round = comm_round
        self.frequency_of_the_test = freq
        self.client_num_per_round = K
        self.client_num_in_total = K


def test_server_manager_sequence_on_a_cpu_server():
    """fedml_server_manager.py:174-251 replayed for three rounds (add xK ->
    check -> aggregate -> test_on_server_for_all_clients -> assess_contribution
    -> client_selection / data_silo_selection): no AttributeError, the
    Context holds the round's client list (fedml_aggregator.py:86) and the
    server metrics of the tested rounds (:193-202), the server model holds
    the average.  The reduction here is the oracle (a CPU server has no
    HBM); tests/test_gpu_cross_silo.py runs the same sequence on the GPU."""
    import copy

    from replay_util import replay_rounds

    from fedml_amd.context import Context
    from fedml_amd.server_aggregator import MI355XServerAggregator
    from fedml_amd.synth import host_clients
    from oracle import fedavg_oracle as orc

    class _OracleAggregator(MI355XServerAggregator):
        def aggregate(self, raw):
            return orc.agg(self.args, raw)

    Context.reset()
    K = 3
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    args = _RoundArgs(K)
    loader, _, _ = _loader()
    server = FedMLAggregator(None, loader, 0, {}, {}, {}, K, torch.device("cpu"), args,
                             _OracleAggregator(model, args))
    assert Context().get(Context.KEY_TEST_DATA) is loader  # :35
    entries = [(k, tuple(t.shape), t.dtype) for k, t in model.state_dict().items()]
    expected = {}

    def updates(r):
        raw = host_clients(entries, K, seed=50 + r, round_idx=r)
        expected[r] = orc.agg(args, copy.deepcopy(raw))
        return raw

    out = replay_rounds(server, args, [11, 12, 13], updates, rounds=3)
    assert args.round_idx == 3
    for o in out:
        r = o["round_idx"]
        assert o["ctx_model_list"] is o["model_list"] and o["idxes"] == [0, 1, 2]
        assert o["ids"] == [11, 12, 13] and o["silos"] == [0, 1, 2]
        for k, e in expected[r].items():
            assert torch.equal(o["global"][k], e)
    # rounds 0 and 2 are tested (freq 2, last round 2); round 1 is not
    m0, m2 = out[0]["metrics"], out[2]["metrics"]
    assert out[1]["metrics"] is m0 and len(m0) == 4 and m0[2] is None
    assert m2 is not m0 and out[2]["metrics_last"] is m0
    for k, e in expected[2].items():
        assert torch.equal(model.state_dict()[k], e)
