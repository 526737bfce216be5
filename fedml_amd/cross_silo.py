"""The cross-silo server's aggregation orchestrator, with client updates
ingested into HBM as they arrive.

Mirrors python/fedml/cross_silo/server/fedml_aggregator.py:13-165 (same
constructor, attribute and method names, argument meaning and return values):

  add_local_trained_result(index, model_params, sample_num)   :58-67
  check_whether_all_receive()                                  :69-76
  aggregate() -> (averaged_params, model_list, idxes)          :78-106
  data_silo_selection / client_selection / client_sampling     :113-165
  test_on_server_for_all_clients(round_idx)                    :177-209

The one behavioural difference is WHERE a client's tensors go on arrival.  The
reference moves them to the server device one tensor at a time
(ml_engine_adapter.model_params_to_device, ml_engine_adapter.py:234-254,
~12 GB/s).  Here the whole update is packed into pinned staging and sent with
one asynchronous H2D per dtype into slot ``index`` of a ``ClientBucket``
(54-56 GB/s, overlapping the next client's arrival), and the dict's values are
rebound to device views of that slot: the same values, dtypes, shapes and
device the reference's dict holds afterwards.  ``aggregate`` is the
reference's, so the server aggregator (FedMLAggOperator.agg on these views:
one multi-tensor launch per key chunk, fedml_amd.agg_operator) and its
on_before / on_after hooks see what they see in FedML.

A slot's views stay valid until that slot receives the next round's update
(the reference's dicts are independent tensors that live on).  Updates the
bucket cannot hold bit-exactly (a key of a dtype other than fp32, bf16, f16,
f64 or int64, a layout different from the first client's) are moved key by key
as in the reference.  The round state goes into FedML's Context registry as
in the reference (fedml_amd.context.shared_context: FedML's own singleton when
FedML is loaded): the test data at construction (:35), the client list of the
round (:86), the server metrics (:197-202), which FedML's contribution
assessment reads back.  Out of scope: mlops logging (plain
logging here) and FHE (an FHE server keeps updates as they arrive, as the
reference does).
"""
from __future__ import annotations

import logging
import random
import time

import numpy as np
import torch

from .agg_operator import _walker, register_resident
from .bucket import ClientBucket
from .context import Context, shared_context
from .layout import ROW_DTYPES
from .multidev import MultiDeviceBucket, devices_for_round, parse_devices


class FedMLAggregator:
    """Same interface as fedml.cross_silo.server.fedml_aggregator.FedMLAggregator."""

    def __init__(self, train_global, test_global, all_train_data_num, train_data_local_dict, test_data_local_dict,
                 train_data_local_num_dict, client_num, device, args, server_aggregator):
        self.aggregator = server_aggregator
        self.args = args
        self.train_global = train_global
        self.test_global = test_global
        self.val_global = self._generate_validation_set()
        self.all_train_data_num = all_train_data_num
        shared_context().add(Context.KEY_TEST_DATA, self.val_global)
        self.train_data_local_dict = train_data_local_dict
        self.test_data_local_dict = test_data_local_dict
        self.train_data_local_num_dict = train_data_local_num_dict
        self.client_num = client_num
        self.device = device
        self.args.device = device
        self.model_dict = dict()
        self.sample_num_dict = dict()
        self.flag_client_model_uploaded_dict = dict()
        for idx in range(self.client_num):
            self.flag_client_model_uploaded_dict[idx] = False
        self.is_fhe_enabled = hasattr(args, "enable_fhe") and args.enable_fhe
        self.bucket = None  # created from the first update's layout
        self._views = {}

    def get_global_model_params(self):
        return self.aggregator.get_model_params()

    def set_global_model_params(self, model_parameters):
        self.aggregator.set_model_params(model_parameters)

    # ---- arrival --------------------------------------------------------------

    def add_local_trained_result(self, index, model_params, sample_num):
        logging.info("add_model. index = %d" % index)
        # :61-63 — a plain dict stays where the user put it; anything else goes
        # to the server device
        if type(model_params) is not dict and (not self.is_fhe_enabled):
            if not self._ingest(index, model_params, sample_num):
                for key in model_params.keys():  # model_params_to_device, key by key
                    model_params[key] = model_params[key].to(self.device)
        self.model_dict[index] = model_params
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

    def _ingest(self, index, model_params, sample_num) -> bool:
        """One H2D per dtype into the bucket slot, then rebind the dict's values
        to device views of it.  False when the bucket cannot hold this update
        exactly (the caller then moves it key by key)."""
        device = torch.device(self.device) if not isinstance(self.device, torch.device) else self.device
        devices = parse_devices(getattr(self.args, "fedagg_devices", None))
        if (device.type != "cuda" and not devices) or not 0 <= index < self.client_num:
            return False
        if device.type != "cuda":
            device = devices[0]
        entries = self._same_layout(model_params)
        if entries is None:  # the first update, or one that may differ: the full check
            entries = []
            for key, t in model_params.items():
                if not isinstance(t, torch.Tensor) or t.dtype not in ROW_DTYPES or t.is_sparse:
                    return False
                entries.append((key, tuple(t.shape), t.dtype))
        if self.bucket is None:
            # int64 keys keep int64 rows, so the views have the update's dtypes.
            # A round that does not fit one GPU (or args.fedagg_devices listing
            # several) is spread over the node's GPUs, whole keys per device:
            # the views are then one-device tensors on different GPUs, and
            # agg() reduces each GPU's keys where they are (fedml_amd.multidev)
            devices = devices_for_round(self.args, entries, self.client_num, device, promote_ints=False)
            if len(devices) > 1:
                self.bucket = MultiDeviceBucket(entries, self.client_num, devices, promote_ints=False)
            else:
                self.bucket = ClientBucket(entries, self.client_num, devices[0], promote_ints=False)
        elif self.bucket.entries != entries:
            return False
        tables = self._walk_one(model_params, entries) if isinstance(self.bucket, ClientBucket) else None
        if tables is not None:
            # one native walk of the dict gives every key's host pointer: the
            # staging pack needs no per-key Python work (config 5's 128 keys
            # per update cost more in Python than its 16.8 MB take on PCIe)
            self.bucket.put_from_table(index, tables, model_params, sample_num, col=0)
        else:
            self.bucket.put(index, model_params, sample_num)
        # work on the current stream (the aggregation, or anything reading the
        # views) is ordered after this slot's H2D; no host synchronisation
        self.bucket.sync_ingest()
        # a slot's views are the same memory every round: built once (320
        # slices cost ~1 ms per ResNet-50 client), then only rebound
        view = self._views.get(index)
        if view is None:
            view = self._views[index] = self.bucket.view(index)
        model_params.update(view)  # the same keys, in the dict's own order
        # agg() over these very dicts then reduces the rows in place
        # (agg_operator._reduce_resident), instead of walking K x keys views
        self.bucket.bind_slot(index, model_params, view)
        register_resident(self.bucket)
        return True

    def _same_layout(self, model_params):
        """The bucket's entries when this update has exactly its keys, shapes
        and dtypes as dense tensors (compared list against list: config 5's
        128 keys cost ~80 us per arrival through the per-key loop), else None."""
        b = self.bucket
        if b is None:
            return None
        sig = getattr(self, "_sig", None)
        if sig is None or sig[0] is not b:
            ents = b.entries
            sig = self._sig = (b, [k for k, _, _ in ents], [torch.Size(s) for _, s, _ in ents],
                               [d for _, _, d in ents])
        vals = list(model_params.values())
        try:
            same = ([t.shape for t in vals] == sig[2] and [t.dtype for t in vals] == sig[3]
                    and list(model_params) == sig[1]
                    and all(isinstance(t, torch.Tensor) and t.layout is torch.strided for t in vals))
        except AttributeError:  # a value without .shape / .dtype
            return None
        return b.entries if same else None

    @staticmethod
    def _walk_one(model_params, entries):
        """The native walker's host pointer tables of this one update
        ({code: int64 [T_code, 1]}), or None when it declines (a device or
        non-contiguous tensor, another dict type, no walker)."""
        w = _walker()
        if w is None:
            return None
        walked = w.walk_host([model_params], [k for k, _, _ in entries])
        if walked is None:
            return None
        _, _, tables = walked
        return {c: np.frombuffer(t, dtype=np.int64).reshape(-1, 1) for c, t in tables.items()}

    def check_whether_all_receive(self):
        logging.debug("client_num = {}".format(self.client_num))
        for idx in range(self.client_num):
            if not self.flag_client_model_uploaded_dict[idx]:
                return False
        for idx in range(self.client_num):
            self.flag_client_model_uploaded_dict[idx] = False
        return True

    # ---- the round --------------------------------------------------------------

    def aggregate(self):
        """:78-106, step for step."""
        start_time = time.time()
        model_list = []
        for idx in range(self.client_num):
            model_list.append((self.sample_num_dict[idx], self.model_dict[idx]))
        model_list, model_list_idxes = self.aggregator.on_before_aggregation(model_list)
        shared_context().add(Context.KEY_CLIENT_MODEL_LIST, model_list)
        averaged_params = self.aggregator.aggregate(model_list)
        if type(averaged_params) is dict:
            if len(averaged_params) == self.client_num + 1:  # {-1: global params} rides along
                itr_count = len(averaged_params) - 1
            else:
                itr_count = len(averaged_params)
            for client_index in range(itr_count):
                averaged_params[client_index] = self.aggregator.on_after_aggregation(averaged_params[client_index])
        else:
            averaged_params = self.aggregator.on_after_aggregation(averaged_params)
        if not self.is_fhe_enabled:
            self.set_global_model_params(averaged_params)
        end_time = time.time()
        logging.info("aggregate time cost: %d" % (end_time - start_time))
        return averaged_params, model_list, model_list_idxes

    def assess_contribution(self):
        if hasattr(self.args, "enable_contribution") and \
                self.args.enable_contribution is not None and self.args.enable_contribution:
            self.aggregator.assess_contribution()

    # ---- server evaluation (:167-209) ----------------------------------------------

    def _generate_validation_set(self, num_samples=10000):
        """:167-175: stackoverflow test sets are subsampled to 10,000 examples."""
        if str(getattr(self.args, "dataset", "")).startswith("stackoverflow"):
            test_data_num = len(self.test_global.dataset)
            sample_indices = random.sample(range(test_data_num), min(num_samples, test_data_num))
            subset = torch.utils.data.Subset(self.test_global.dataset, sample_indices)
            return torch.utils.data.DataLoader(subset, batch_size=self.args.batch_size)
        return self.test_global

    def test_on_server_for_all_clients(self, round_idx):
        """:177-209, called by FedMLServerManager after every aggregate()
        (fedml_server_manager.py:202): every `frequency_of_the_test` rounds and
        on the last one, evaluate the aggregated model (the full test set on
        the last round, the validation set otherwise) and record the metrics
        and the previous round's in the Context."""
        if self.is_fhe_enabled:
            logging.info("Encrypted global model cannot be tested on the server")
            return
        if round_idx % self.args.frequency_of_the_test == 0 or round_idx == self.args.comm_round - 1:
            logging.info("################test_on_server_for_all_clients : {}".format(round_idx))
            self.aggregator.test_all(self.train_data_local_dict, self.test_data_local_dict, self.device, self.args)
            if round_idx == self.args.comm_round - 1:
                metric_result_in_current_round = self.aggregator.test(self.test_global, self.device, self.args)
            else:
                metric_result_in_current_round = self.aggregator.test(self.val_global, self.device, self.args)
            logging.info("metric_result_in_current_round = {}".format(metric_result_in_current_round))
            ctx = shared_context()
            metric_results_in_the_last_round = ctx.get(Context.KEY_METRICS_ON_AGGREGATED_MODEL)
            ctx.add(Context.KEY_METRICS_ON_AGGREGATED_MODEL, metric_result_in_current_round)
            if metric_results_in_the_last_round is not None:
                ctx.add(Context.KEY_METRICS_ON_LAST_ROUND, metric_results_in_the_last_round)
            else:
                ctx.add(Context.KEY_METRICS_ON_LAST_ROUND, metric_result_in_current_round)
            logging.info("key_metrics_on_last_round = {}".format(ctx.get(Context.KEY_METRICS_ON_LAST_ROUND)))
        logging.info("round_idx = %d" % round_idx)  # mlops.log({"round_idx": ...}) in the reference

    # ---- model-serving metadata (:211-258) -------------------------------------------

    def _dummy_features(self):
        """First sample of the first batch of the server's test loader (or of
        the first non-empty client test loader when there is none), every
        tensor of the batch but the last (the label), as the reference does."""
        loader = self.test_global
        if not loader:
            for _, v in self.test_data_local_dict.items():
                if v:
                    loader = v
                    break
        with torch.no_grad():
            batch = next(iter(loader))
            firsts = [t[:1] for t in batch]
        return firsts[:-1]

    def get_dummy_input_tensor(self):
        """:211-227, called by FedMLServerManager before the first round
        (fedml_server_manager.py:71-85) to log the model's input for serving."""
        return self._dummy_features()

    def get_input_shape_type(self):
        """:229-258: per input feature its shape and "int" for integer / bool
        dtypes, "float" otherwise."""
        ints = (torch.int8, torch.int16, torch.int32, torch.int64, torch.uint8, torch.bool)
        shapes, types = [], []
        for f in self._dummy_features():
            shapes.append(list(f.shape))
            types.append("int" if f.dtype in ints else "float")
        return shapes, types

    # ---- client selection (:113-165, the same seeded numpy draws) ------------------

    def data_silo_selection(self, round_idx, client_num_in_total, client_num_per_round):
        logging.info("client_num_in_total = %d, client_num_per_round = %d" % (client_num_in_total,
                                                                              client_num_per_round))
        assert client_num_in_total >= client_num_per_round
        if client_num_in_total == client_num_per_round:
            return [i for i in range(client_num_per_round)]
        np.random.seed(round_idx)
        return np.random.choice(range(client_num_in_total), client_num_per_round, replace=False)

    def client_selection(self, round_idx, client_id_list_in_total, client_num_per_round):
        if client_num_per_round == len(client_id_list_in_total):
            return client_id_list_in_total
        np.random.seed(round_idx)
        return np.random.choice(client_id_list_in_total, client_num_per_round, replace=False)

    def client_sampling(self, round_idx, client_num_in_total, client_num_per_round):
        if client_num_in_total == client_num_per_round:
            client_indexes = [client_index for client_index in range(client_num_in_total)]
        else:
            num_clients = min(client_num_per_round, client_num_in_total)
            np.random.seed(round_idx)
            client_indexes = np.random.choice(range(client_num_in_total), num_clients, replace=False)
        logging.info("client_indexes = %s" % str(client_indexes))
        return client_indexes
