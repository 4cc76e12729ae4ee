"""Coverage metrics (reference ``recommenders/evaluate/coverage.py:4-74``),
fed from top-k index matrices instead of (B, A) predictions."""
import numpy as np
import torch


def get_coverage_k(unique_topk_actions, unpopular_items, num_actions):
    assert isinstance(unique_topk_actions, set) and isinstance(unpopular_items, set)
    unpopular_coverage = len(unique_topk_actions & unpopular_items) / len(unpopular_items)
    return unpopular_coverage, len(unique_topk_actions) / num_actions


def update_coverage_from_indices(idx, actions_covered_topk_dict, top_k):
    """Add every row's first k ids to the covered set of each k (reference
    update_actions_covered_topk_dict, coverage.py:24-53).  The batch's ids are
    de-duplicated first and the covered set is grown in place (O(batch)
    instead of the reference's O(|covered|) ``union`` copy per batch; the
    dict ends up holding the same sets)."""
    idx = np.asarray(idx)
    for k in top_k:
        new = np.unique(idx[:, :k]).tolist()
        cur = actions_covered_topk_dict[k]
        if isinstance(cur, set):
            cur.update(new)
        else:
            actions_covered_topk_dict[k] = set(cur).union(new)
    return actions_covered_topk_dict


def update_actions_covered_topk_dict(predictions, actions_covered_topk_dict, top_k, input_tokenizer=None,
                                     output_tokenizer=None):
    _, top = torch.topk(predictions, k=max(top_k))
    return update_coverage_from_indices(top.cpu().numpy(), actions_covered_topk_dict, top_k)


def get_coverage(actions_covered_topk_dict, unpopular_set, num_actions, topk):
    return {k: get_coverage_k(actions_covered_topk_dict[k], unpopular_set, num_actions) for k in topk}
