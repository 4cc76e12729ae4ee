"""Q-head tensor helpers (reference ``recommenders/utils/tensor_operations.py:4-84``).

The MI355X training step never materialises the (B, heads, A) Q tensor: the
same math runs as ``rg_q_gather`` (gather_from_3d at the taken / target
action), ``rg_weighted_sum`` + the fused GEMM-argmax (get_weighted_q_target +
get_max_action) and ``rg_smorl_td`` (weighted_q_loss).  These functions keep
the reference's tensor API for external callers."""
import torch


def gather_from_3d(q_tensor, action_idxs, num_heads):
    """(B, heads, A), (B,) -> (B, heads): every head's value at each row's action."""
    ix = action_idxs.view(-1, 1, 1).expand(-1, num_heads, 1)
    return torch.gather(q_tensor, dim=2, index=ix).squeeze()


def weighted_q_loss(q_vals, w):
    """(B, heads) x (heads,) -> (B,)."""
    return torch.matmul(q_vals, w)


def get_weighted_q_target(q_vals, w):
    """sum_i w_i Q_i over the head axis -> (B, A)."""
    return torch.sum(q_vals * w.to(q_vals.device).view(1, -1, 1), dim=1)


def get_max_action(q_vals):
    return torch.argmax(q_vals, dim=1)
