"""The process-wide registry FedML's server writes round state into.

Mirrors python/fedml/core/alg_frame/context.py:19-39 (a Params singleton,
params.py:1-29, singleton.py:1-5): the same key names and add/get semantics
(``get`` of an absent key is None).  The cross-silo aggregator registers the
round's client list under KEY_CLIENT_MODEL_LIST (fedml_aggregator.py:86) and
the server metrics under KEY_METRICS_ON_* (:197-202); contribution assessment
reads them back (server_aggregator.py:109-117).

``shared_context()`` is what the mirrors call: when FedML itself is loaded in
the process (the drop-in case) it returns FedML's own Context
singleton, so FedML's server manager and contribution code see the entries;
otherwise this module's singleton.
"""
from __future__ import annotations

import sys


class Params:
    """params.py:1-29: attribute bag with add/get/keys/values."""

    KEY_MODEL_PARAMS = "model_params"

    def __init__(self, **kwargs):
        self.__dict__.update(kwargs)

    def add(self, name: str, value) -> None:
        self.__dict__[name] = value

    def get(self, name: str):
        if not hasattr(self, name):
            return None
        return getattr(self, name)

    def keys(self):
        return self.__dict__.keys()

    def values(self):
        return self.__dict__.values()


class Context(Params):
    """context.py:19-39: one instance per process (Context() is Context())."""

    KEY_CLIENT_ID_LIST_IN_THIS_ROUND = "client_id_list_in_this_round"
    KEY_TEST_DATA = "test_data"
    KEY_CLIENT_MODEL_LIST = "client_model_list"
    KEY_RECEIVED_MODEL_CID = "received_model_cid"
    KEY_SENT_MODEL_CID = "sent_model_cid"
    KEY_METRICS_ON_LAST_ROUND = "metrics_on_last_round"
    KEY_METRICS_ON_AGGREGATED_MODEL = "metrics_on_aggregated_model"
    KEY_IPFS_SECRET_KEY = "ipfs_secret_key"

    def __new__(cls, *args, **kw):
        if "_instance" not in cls.__dict__:
            cls._instance = super().__new__(cls)
        return cls._instance

    def __init__(self, **kwargs):
        super().__init__(**kwargs)

    @classmethod
    def reset(cls) -> None:
        """Drop every entry (tests; FedML has no equivalent, one run per process)."""
        inst = cls.__dict__.get("_instance")
        if inst is not None:
            inst.__dict__.clear()


def shared_context():
    """FedML's Context when FedML is loaded in this process, else ours."""
    mod = sys.modules.get("fedml.core.alg_frame.context")
    ctx_cls = getattr(mod, "Context", None) if mod is not None else None
    return ctx_cls() if ctx_cls is not None else Context()
