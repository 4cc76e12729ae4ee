"""Diversity reward (reference ``recommenders/evaluate/diversity.py:4-73``).

The training step and the evaluator compute it with the ``rg_diversity``
kernel on device top-k indices; these functions keep the reference's tensor
API for callers that hold (B, A) predictions."""
import torch


def map_ids_host(idx, input_tokenizer, output_tokenizer):
    """input_tokenizer.stoi(output_tokenizer.itos(x)) for every element (the
    reference's apply_ branch) through the pair's cached lookup table
    (recommenders/hip/remap.py host_table); an id with no input token raises
    KeyError (RemapError) as the reference's stoi does."""
    from recommenders.hip.remap import RemapError, host_table
    lut = host_table(input_tokenizer, output_tokenizer)
    i = idx.cpu().long()
    if bool(((i < 0) | (i >= len(lut))).any()):
        raise IndexError("predicted id outside the output vocabulary")
    out = lut[i].long()
    if bool((out < 0).any()):
        raise RemapError("a predicted id has no input-vocabulary token (input_tokenizer.stoi(output_tokenizer.itos(id)))")
    return out.to(idx.device)


def get_last_action(s, padding_pos, s_len=None, device="cuda"):
    if padding_pos == "end":
        idx = s_len.to(s.device) - 1
        return s.gather(index=idx.unsqueeze(1), dim=1).squeeze(1)
    return s[:, -1]


def get_batch_diversity_rewards(s, predictions, len_states, padding_pos, topk_to_consider, embedding_layer,
                                device="cuda", input_tokenizer=None, output_tokenizer=None):
    """1 - mean_k cos(E[last action], E[top-k prediction]) per row (eps 1e-6)."""
    last = get_last_action(s, padding_pos, len_states, device)
    _, idx = torch.topk(predictions, k=topk_to_consider)
    if input_tokenizer is not None:   # output -> input vocabulary (tabulated, recommenders/hip/remap.py)
        idx = map_ids_host(idx, input_tokenizer, output_tokenizer)
    e_last = embedding_layer(last.to(idx.device)).unsqueeze(1)
    e_pred = embedding_layer(idx)
    sim = torch.nn.functional.cosine_similarity(e_last, e_pred, dim=2, eps=1e-6)
    return 1 - torch.mean(sim, dim=1)
