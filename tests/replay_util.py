"""Replays FedMLServerManager.handle_message_receive_model_from_client
(python/fedml/cross_silo/server/fedml_server_manager.py:174-251) against the
cross-silo aggregator mirror, without the transport: the exact sequence of
aggregator calls a FedML server makes every round."""
from __future__ import annotations

from fedml_amd.context import Context, shared_context


def replay_rounds(aggregator, args, client_real_ids, updates_for_round, rounds):
    """updates_for_round(round_idx) -> [(sample_num, state_dict)] in the
    order of client_real_ids.  Returns, per round, what the manager would
    broadcast and the bookkeeping it reads."""
    ctx = shared_context()
    client_id_list_in_this_round = list(client_real_ids[:args.client_num_per_round])
    out = []
    for _ in range(rounds):
        updates = updates_for_round(args.round_idx)
        b_all_received = False
        for sender_id, (n, params) in zip(client_id_list_in_this_round, updates):  # :174-185
            aggregator.add_local_trained_result(client_real_ids.index(sender_id), params, n)
            b_all_received = aggregator.check_whether_all_receive()
        assert b_all_received
        global_model_params, model_list, model_list_idxes = aggregator.aggregate()  # :190
        new_ids = [client_id_list_in_this_round[i] for i in model_list_idxes]  # :193-197
        ctx.add(Context.KEY_CLIENT_ID_LIST_IN_THIS_ROUND, new_ids)
        aggregator.test_on_server_for_all_clients(args.round_idx)  # :202
        aggregator.assess_contribution()  # :204
        client_id_list_in_this_round = aggregator.client_selection(  # :211-216
            args.round_idx, client_real_ids, args.client_num_per_round)
        data_silo_index_list = aggregator.data_silo_selection(
            args.round_idx, args.client_num_in_total, len(client_id_list_in_this_round))
        ctx.add(Context.KEY_CLIENT_ID_LIST_IN_THIS_ROUND, client_id_list_in_this_round)
        out.append({
            "round_idx": args.round_idx,
            "global": global_model_params,
            "model_list": model_list,
            "idxes": model_list_idxes,
            "metrics": ctx.get(Context.KEY_METRICS_ON_AGGREGATED_MODEL),
            "metrics_last": ctx.get(Context.KEY_METRICS_ON_LAST_ROUND),
            "ctx_model_list": ctx.get(Context.KEY_CLIENT_MODEL_LIST),
            "silos": list(data_silo_index_list),
            "ids": list(client_id_list_in_this_round),
        })
        args.round_idx += 1  # :245
    return out
