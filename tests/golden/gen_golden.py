"""Generate golden vectors by running the REFERENCE aggregator (CPU container).

    python tests/golden/gen_golden.py [case-name-prefix ...]

Imports FedML's own code from /root/reference/python (read-only) through
namespace-package stubs, so only the modules on the aggregation path load:

  fedml.ml.aggregator.agg_operator.FedMLAggOperator     agg_operator.py:8-234
  fedml.simulation.mpi.fedopt.FedOptAggregator          FedOptAggregator.py:14-130
  (+ its optrepo; `wandb` is absent and replaced by an empty module)

For each case of tests/golden/cases.py it records the sha256 of the inputs,
the reference's outputs (bit patterns), the exception type it raises, and the
aliasing it exhibits.  Only data is written (tests/golden/fixtures/*.npz, no
pickles); no reference source is copied.  The GPU box never runs this file.
"""
from __future__ import annotations

import json
import os
import sys
import types
from collections import OrderedDict

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import cases  # noqa: E402
from fedml_amd.synth import fingerprint  # noqa: E402

REF = "/root/reference/python/fedml"
OUT_DIR = os.path.join(HERE, "fixtures")


def import_reference():
    for name, path in [
        ("fedml", REF), ("fedml.core", f"{REF}/core"), ("fedml.simulation", f"{REF}/simulation"),
        ("fedml.simulation.mpi", f"{REF}/simulation/mpi"),
        ("fedml.simulation.mpi.fedopt", f"{REF}/simulation/mpi/fedopt"),
    ]:
        m = types.ModuleType(name)
        m.__path__ = [path]
        sys.modules[name] = m
    sys.modules.setdefault("wandb", types.ModuleType("wandb"))
    from fedml.ml.aggregator.agg_operator import FedMLAggOperator
    from fedml.simulation.mpi.fedopt.FedOptAggregator import FedOptAggregator
    return FedMLAggOperator, FedOptAggregator


def import_defenses():
    for name, path in [("fedml.core.security", f"{REF}/core/security"),
                       ("fedml.core.security.defense", f"{REF}/core/security/defense"),
                       ("fedml.core.security.common", f"{REF}/core/security/common")]:
        m = types.ModuleType(name)
        m.__path__ = [path]
        sys.modules[name] = m
    from fedml.core.security.defense.coordinate_wise_median_defense import CoordinateWiseMedianDefense
    from fedml.core.security.defense.coordinate_wise_trimmed_mean_defense import CoordinateWiseTrimmedMeanDefense
    return CoordinateWiseMedianDefense, CoordinateWiseTrimmedMeanDefense


class _Done(Exception):
    """Carries a finished defense's result out of run_dist_case's try block."""

    def __init__(self, res):
        super().__init__("done")
        self.res = res


def run_dist_case(FedMLAggOperator, spec):
    """Krum / multi-Krum / norm-diff clipping through the reference's own
    classes (krum_defense.py, norm_diff_clipping_defense.py), then the base
    FedAvg operator.  Records the returned list (which input tuples Krum kept,
    in order; every clipped dict), the reference's own Krum scores and
    clipping norms, and the aggregated model."""
    from fedml.core.security.common import utils as sec_utils
    from fedml.core.security.defense.krum_defense import KrumDefense
    from fedml.core.security.defense.norm_diff_clipping_defense import NormDiffClippingDefense

    raw, glob = cases.dist_inputs(spec)
    args = cases.DefenseArgs(spec)
    meta = {"spec": spec, "in_sha256": fingerprint(raw), "error": None, "tuple": False}
    arrays = {}
    ids = [id(item) for item in raw]
    try:
        if spec["defense"] == "robust_learning_rate":
            from fedml.core.security.defense.robust_learning_rate_defense import RobustLearningRateDefense

            d = RobustLearningRateDefense(args)
            res = d.run(raw, lambda lst: FedMLAggOperator.agg(args, lst))
            meta["returns_client0_dict"] = res is raw[0][1]
            raise _Done(res)
        if spec["defense"] == "slsgd":
            from fedml.core.security.defense.slsgd_defense import SLSGDDefense

            d = SLSGDDefense(args)
            lst = d.defend_before_aggregation(raw, glob)
            dict_ids = [id(item[1]) for item in raw]  # trimmed_mean builds new tuples around the same dicts
            meta["selected"] = [dict_ids.index(id(item[1])) for item in lst]
            for k, t in glob.items():
                arrays[f"g:{k}"] = tensor_bytes(t)
            res = d.defend_on_aggregation(lst, FedMLAggOperator.agg, glob)
            raise _Done(res)
        if spec["defense"] == "cclip":
            from fedml.core.security.defense.cclip_defense import CClipDefense

            d = CClipDefense(args)
            np.random.seed(spec["np_seed"])
            lst = d.defend_before_aggregation(raw, None)
            B = len(lst)
            np.random.seed(spec["np_seed"])
            meta["guess_index"] = int(np.random.randint(0, B))
            meta["bucket_nums"] = [float(n) for n, _ in lst]
            for b, (_, dct) in enumerate(lst):
                for k, t in dct.items():
                    arrays[f"c{b}:{k}"] = tensor_bytes(t)
            res = d.defend_after_aggregation(FedMLAggOperator.agg(args, lst))
            raise _Done(res)
        if spec["defense"] in ("krum", "multikrum"):
            d = KrumDefense(args)
            vecs = [sec_utils.vectorize_weight(p) for _, p in raw]
            meta["ref_scores"] = [float(x) for x in d._compute_krum_score(vecs)]
            out_list = d.defend_before_aggregation(raw, None)
            meta["selected"] = [ids.index(id(item)) for item in out_list]
        else:
            d = NormDiffClippingDefense(args)
            vg = sec_utils.vectorize_weight(glob)
            meta["ref_norms"] = [float(torch.norm(sec_utils.vectorize_weight(p) - vg).item()) for _, p in raw]
            out_list = d.defend_before_aggregation(raw, glob)
            for i, (_, dct) in enumerate(out_list):
                for k, t in dct.items():
                    arrays[f"c{i}:{k}"] = tensor_bytes(t)
            for k, t in glob.items():
                arrays[f"g:{k}"] = tensor_bytes(t)
        res = FedMLAggOperator.agg(args, out_list)
    except _Done as dn:
        res = dn.res
    except Exception as e:
        meta["error"] = type(e).__name__
        save(spec["name"], meta, arrays)
        return
    meta["outputs"] = []
    for k, t in res.items():
        arrays[f"o0:{k}"] = tensor_bytes(t)
        meta["outputs"].append({"group": 0, "key": k, "dtype": str(t.dtype).replace("torch.", ""),
                                "shape": list(t.shape), "is_client0_tensor": False})
    save(spec["name"], meta, arrays)


def tensor_bytes(t: torch.Tensor) -> np.ndarray:
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16).copy()
    if t.dtype == torch.bool:
        return t.numpy().astype(np.uint8)
    return t.numpy().copy()


def save(name: str, meta: dict, arrays: dict) -> None:
    os.makedirs(OUT_DIR, exist_ok=True)
    payload = {f"a{i}": v for i, v in enumerate(arrays.values())}
    meta["array_names"] = list(arrays.keys())
    np.savez_compressed(os.path.join(OUT_DIR, f"{name}.npz"), meta=np.array(json.dumps(meta)), **payload)


def run_agg_case(FedMLAggOperator, spec, aggregate=None):
    raw = cases.build_inputs(spec)
    sha = fingerprint(raw)
    client0_before = OrderedDict((k, t.clone()) for k, t in raw[0][1].items())
    client0_objs = dict(raw[0][1])
    # 3-tuple optimizers (SCAFFOLD, Mime): client 0's second dict too
    # (SCAFFOLD's `total_c_delta_para[k] += c_delta_para[k]` adds into its tensors)
    third_before = OrderedDict((k, t.clone()) for k, t in raw[0][2].items()) if len(raw[0]) > 2 else None
    third_objs = dict(raw[0][2]) if len(raw[0]) > 2 else None
    meta = {"spec": spec, "in_sha256": sha, "error": None}
    arrays = {}
    try:
        res = aggregate(raw) if aggregate is not None else FedMLAggOperator.agg(cases.Args(spec), raw)
    except Exception as e:  # the reference's own error behaviour is part of the contract
        meta["error"] = type(e).__name__
        save(spec["name"], meta, arrays)
        return
    groups = list(res) if isinstance(res, tuple) else [res]
    meta["tuple"] = isinstance(res, tuple)
    meta["result_is_client0_dict"] = groups[0] is raw[0][1]
    meta["outputs"] = []
    for g, d in enumerate(groups):
        for k, t in d.items():
            arrays[f"o{g}:{k}"] = tensor_bytes(t)
            meta["outputs"].append({"group": g, "key": k, "dtype": str(t.dtype).replace("torch.", ""),
                                    "shape": list(t.shape),
                                    "is_client0_tensor": (k in client0_objs and t is client0_objs[k])})
    mutated = [k for k, t in client0_objs.items()
               if not torch.equal(t.view(torch.int16) if t.dtype == torch.bfloat16 else t,
                                  client0_before[k].view(torch.int16) if t.dtype == torch.bfloat16
                                  else client0_before[k])
               and not (t.is_floating_point() and torch.isnan(t).any())]
    meta["client0_tensors_mutated"] = mutated
    if third_objs is not None:
        mutated2 = [k for k, t in third_objs.items() if not torch.equal(t, third_before[k])
                    and not (t.is_floating_point() and torch.isnan(t).any())]
        meta["client0_third_tensors_mutated"] = mutated2
        for k in mutated2:  # the mutated tensors' values after the call
            arrays[f"m2:{k}"] = tensor_bytes(third_objs[k])
    save(spec["name"], meta, arrays)


def run_fedopt_case(FedOptAggregator, spec):
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(10, 5), torch.nn.BatchNorm1d(5), torch.nn.Linear(5, 3))
    model.load_state_dict(cases.fedopt_global_init(spec))

    class ServerAgg:
        def __init__(self, m):
            self.model = m

        def get_model_params(self):
            return self.model.state_dict()

        def set_model_params(self, sd):
            self.model.load_state_dict(sd)

    class A:
        server_optimizer = "sgd"
        server_lr = spec["lr"]
        server_momentum = spec["momentum"]

    agg = object.__new__(FedOptAggregator)
    agg.aggregator = ServerAgg(model)
    agg.args = A()
    agg.worker_num = spec["K"]
    agg.model_dict, agg.sample_num_dict, agg.flag_client_model_uploaded_dict = {}, {}, {}
    agg.opt = agg._instantiate_opt()
    meta = {"spec": spec, "rounds": [], "param_names": cases.FEDOPT_PARAMS}
    arrays = {}
    for k, t in cases.fedopt_global_init(spec).items():
        arrays[f"init:{k}"] = tensor_bytes(t)
    gsd = OrderedDict((k, t.clone()) for k, t in model.state_dict().items())
    for r in range(spec["rounds"]):
        raw = cases.fedopt_round_inputs(spec, gsd, r)
        meta["rounds"].append({"in_sha256": fingerprint(raw)})
        for j in spec.get("alias_of_0", ()):  # the same dict object at index j as at index 0
            raw[j] = (raw[j][0], raw[0][1])
        for i, (n, d) in enumerate(raw):
            agg.add_local_trained_result(i, d, n)
        out = agg.aggregate()
        gsd = OrderedDict((k, t.detach().clone()) for k, t in out.items())
        for k, t in gsd.items():
            arrays[f"r{r}:{k}"] = tensor_bytes(t)
    save(spec["name"], meta, arrays)


# torch's per-parameter state recorded per round (scalar tensors included)
STATE_BUFFERS = {"adagrad": ("sum",), "rmsprop": ("square_avg",), "adamax": ("exp_avg", "exp_inf"),
                 "nadam": ("exp_avg", "exp_avg_sq", "mu_product"), "radam": ("exp_avg", "exp_avg_sq"),
                 "adadelta": ("square_avg", "acc_delta"), "asgd": ("ax", "eta", "mu"),
                 "rprop": ("prev", "step_size")}


def import_sp_fedopt():
    """sp/fedopt/fedopt_api.py's FedOptAPI (its trainer factory import is stubbed:
    only _aggregate / _set_model_global_grads / _instanciate_opt are used)."""
    for name, path in [("fedml.simulation.sp", f"{REF}/simulation/sp"),
                       ("fedml.simulation.sp.fedopt", f"{REF}/simulation/sp/fedopt")]:
        m = types.ModuleType(name)
        m.__path__ = [path]
        sys.modules.setdefault(name, m)
    if "fedml.ml.trainer" not in sys.modules:  # its __init__ pulls in every trainer
        m = types.ModuleType("fedml.ml.trainer")
        m.__path__ = []
        sys.modules["fedml.ml.trainer"] = m
    tc = types.ModuleType("fedml.ml.trainer.trainer_creator")
    tc.create_model_trainer = None
    sys.modules["fedml.ml.trainer.trainer_creator"] = tc
    from fedml.simulation.sp.fedopt.fedopt_api import FedOptAPI
    return FedOptAPI


def run_fedopt_adam_case(FedOptAPI, spec):
    """The server half of FedOptAPI.train (fedopt_api.py:121-130) with
    server_optimizer="adam" (or spec["optimizer"], e.g. "adagrad"): _aggregate, then zero_grad / state_dict /
    _set_model_global_grads / _instanciate_opt / load_state_dict / step, each the
    reference's own method.  Clients are the synthetic updates of cases.py."""
    ent = cases.FEDOPT_MODELS[spec["model"]]
    dims = [ent[0][1][1], ent[0][1][0], ent[7][1][0]]
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(dims[0], dims[1]), torch.nn.BatchNorm1d(dims[1]),
                                torch.nn.Linear(dims[1], dims[2]))
    model.load_state_dict(cases.fedopt_global_init(spec))

    class Trainer:
        def __init__(self, m):
            self.model = m

        def get_model_params(self):
            return self.model.state_dict()

        def set_model_params(self, sd):
            self.model.load_state_dict(sd)

    class A:
        server_optimizer = spec.get("optimizer", "adam")
        server_lr = spec["lr"]

    if A.server_optimizer == "adamw":
        # torch.optim.AdamW subclasses Adam, so OptRepo (direct subclasses of
        # Optimizer only, optrepo.py:10) cannot name it and the reference
        # raises KeyError.  The fixture runs the same FedOptAPI flow with AdamW
        # registered, i.e. torch's AdamW as FedOptAPI would drive it.
        from fedml.simulation.sp.fedopt.optrepo import OptRepo

        OptRepo.repo.setdefault("adamw", torch.optim.AdamW)
    api = object.__new__(FedOptAPI)
    api.args = A()
    api.model_trainer = Trainer(model)
    api._instanciate_opt()
    meta = {"spec": spec, "rounds": [], "param_names": cases.FEDOPT_PARAMS}
    arrays = {}
    for k, t in cases.fedopt_global_init(spec).items():
        arrays[f"init:{k}"] = tensor_bytes(t)
    gsd = OrderedDict((k, t.clone()) for k, t in model.state_dict().items())
    for r in range(spec["rounds"]):
        raw = cases.fedopt_round_inputs(spec, gsd, r)
        meta["rounds"].append({"in_sha256": fingerprint(raw)})
        w_avg = api._aggregate(raw)
        api.opt.zero_grad()
        opt_state = api.opt.state_dict()
        api._set_model_global_grads(w_avg)
        api._instanciate_opt()
        api.opt.load_state_dict(opt_state)
        api.opt.step()
        gsd = OrderedDict((k, t.detach().clone()) for k, t in model.state_dict().items())
        for k, t in gsd.items():
            arrays[f"r{r}:{k}"] = tensor_bytes(t)
        st = api.opt.state_dict()["state"]
        for j, name in enumerate(cases.FEDOPT_PARAMS):
            for buf in STATE_BUFFERS.get(A.server_optimizer, ("exp_avg", "exp_avg_sq")):
                arrays[f"r{r}:{buf}:{name}"] = tensor_bytes(st[j][buf])
    save(spec["name"], meta, arrays)


def run_secagg_case(spec):
    """The reference's own aggregate_models_in_finite / aggregate_model_reconstruction."""
    for name, path in [("fedml.core.mpc", f"{REF}/core/mpc"), ("fedml.cross_silo", f"{REF}/cross_silo"),
                       ("fedml.cross_silo.lightsecagg", f"{REF}/cross_silo/lightsecagg")]:
        m = types.ModuleType(name)
        m.__path__ = [path]
        sys.modules.setdefault(name, m)
    sys.modules.setdefault("fedml.mlops", types.ModuleType("fedml.mlops"))
    sys.modules["fedml"].mlops = sys.modules["fedml.mlops"]
    from fedml.core.mpc.lightsecagg import aggregate_models_in_finite, model_dimension
    from fedml.cross_silo.lightsecagg.lsa_fedml_aggregator import LightSecAggAggregator

    dicts, mask = cases.secagg_inputs(spec)
    meta = {"spec": spec, "error": None, "tuple": False}
    arrays = {}
    if spec["kind"] == "finite_sum":
        out = aggregate_models_in_finite(dicts, spec["p"])
        res = OrderedDict((k, torch.from_numpy(np.asarray(v))) for k, v in out.items())
    else:
        agg = object.__new__(LightSecAggAggregator)
        agg.model_dict = {i: d for i, d in enumerate(dicts)}
        agg.dimensions, _ = model_dimension(OrderedDict((k, torch.from_numpy(v)) for k, v in dicts[0].items()))
        agg.prime_number = spec["p"]
        agg.precision_parameter = spec["q"]
        agg.aggregate_mask_reconstruction = lambda active: mask
        agg.set_global_model_params = lambda params: None
        res = agg.aggregate_model_reconstruction(list(range(spec["K"])), list(range(spec["K"])))
    meta["outputs"] = []
    for k, t in res.items():
        arrays[f"o0:{k}"] = tensor_bytes(t)
        meta["outputs"].append({"group": 0, "key": k, "dtype": str(t.dtype).replace("torch.", ""),
                                "shape": list(t.shape), "is_client0_tensor": False})
    save(spec["name"], meta, arrays)


def import_mpi_fedavg():
    """simulation/mpi/fedavg/FedAVGAggregator.py with its module-level imports
    stubbed: wandb, fedml.mlops, and the attacker / defender singletons (only
    _fedavg_aggregation_ runs; it touches none of them)."""
    for name, path in [("fedml.simulation.mpi.fedavg", f"{REF}/simulation/mpi/fedavg"),
                       ("fedml.core.security", f"{REF}/core/security")]:
        m = types.ModuleType(name)
        m.__path__ = [path]
        sys.modules.setdefault(name, m)
    sys.modules.setdefault("fedml.mlops", types.ModuleType("fedml.mlops"))
    sys.modules["fedml"].mlops = sys.modules["fedml.mlops"]
    for mod, cls in [("fedml.core.security.fedml_attacker", "FedMLAttacker"),
                     ("fedml.core.security.fedml_defender", "FedMLDefender")]:
        if mod not in sys.modules:
            m = types.ModuleType(mod)
            setattr(m, cls, type(cls, (), {}))
            sys.modules[mod] = m
    from fedml.simulation.mpi.fedavg.FedAVGAggregator import FedAVGAggregator
    return FedAVGAggregator


def main(only=()):
    """only: case-name prefixes to regenerate (default: every case)."""
    def want(spec):
        return not only or any(spec["name"].startswith(p) for p in only)

    FedMLAggOperator, FedOptAggregator = import_reference()
    for spec in filter(want, cases.CASES + cases.ALIAS_CASES):
        run_agg_case(FedMLAggOperator, spec)
        print("wrote", spec["name"])
    for spec in filter(want, cases.FEDOPT_CASES + cases.FEDOPT_ALIAS_CASES):
        run_fedopt_case(FedOptAggregator, spec)
        print("wrote", spec["name"])
    FedOptAPI = import_sp_fedopt()
    for spec in filter(want, cases.FEDOPT_ADAM_CASES + cases.FEDOPT_ADAGRAD_CASES + cases.FEDOPT_ADAMW_CASES
                       + cases.FEDOPT_RMSPROP_CASES + cases.FEDOPT_OPTREPO_CASES):
        run_fedopt_adam_case(FedOptAPI, spec)
        print("wrote", spec["name"])
    Median, Trimmed = import_defenses()
    for spec in filter(want, cases.DEFENSE_CASES):
        args = cases.DefenseArgs(spec)
        if spec["defense"] == "wise_median":
            # FedMLDefender.defend_on_aggregation -> CoordinateWiseMedianDefense (fedml_defender.py:163-171)
            def agg(raw, args=args):
                return Median(args).defend_on_aggregation(raw, FedMLAggOperator.agg, None)
        else:
            # defend_before_aggregation -> trimmed list, then the base FedAvg operator
            def agg(raw, args=args):
                return FedMLAggOperator.agg(args, Trimmed(args).defend_before_aggregation(raw, None))
        run_agg_case(FedMLAggOperator, spec, aggregate=agg)
        print("wrote", spec["name"])
    for spec in filter(want, cases.DIST_CASES):
        run_dist_case(FedMLAggOperator, spec)
        print("wrote", spec["name"])
    for spec in filter(want, cases.SECAGG_CASES):
        run_secagg_case(spec)
        print("wrote", spec["name"])
    mpi = [spec for spec in cases.MPI_CASES if want(spec)]
    if mpi:
        FedAVGAggregator = import_mpi_fedavg()
        agg = object.__new__(FedAVGAggregator)
        for spec in mpi:
            run_agg_case(FedMLAggOperator, spec, aggregate=agg._fedavg_aggregation_)
            print("wrote", spec["name"])


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))
