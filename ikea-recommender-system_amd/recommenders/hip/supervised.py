"""One supervised (full-softmax CE) training step on the MI355X — the shared
body of GRU4Rec_trainer and BidirGRU4Rec_trainer
(GRU4Rec/model.py:129-155, BidirGRU4Rec/model.py:150-176):

  pack -> gather -> W_ih GEMM -> GRU recurrence -> [dropout] -> logits + online
  LSE -> CE loss -> dh (split-K) + fused dW/db/Adam of the head -> BPTT ->
  dX / dW_ih / dW_hh / bias sums -> embedding scatter -> Adam sweeps.
"""
from __future__ import annotations


import torch

from .hostsync import InputStage
from .nets import HipNet


class SupervisedNet(HipNet):
    def forward(self, s, lengths):
        if self.comm is not None:
            raise NotImplementedError("forward() of an item-sharded model: each rank holds a slice of the items")
        h = self.hidden(s, lengths, slot="eval", save=False)
        if self.training and self.dropout_p > 0:
            mask = self.dropout_mask(h.shape[0])
            h = self.apply_mask(h, mask, torch.empty_like(h))
        head = next(iter(self.heads.values()))
        _, z = head.logits_T(h)
        return z




def supervised_step(net: SupervisedNet, clock, s, a, true_len, host=None):
    """Returns the device loss tensor (1,) — the caller does the .item(), or,
    with ``host`` (hostsync.HostScalars), reads the loss captured as soon as
    it is final."""
    dev = net.device
    if getattr(net, "_inputs", None) is None:
        net._inputs = InputStage(dev)
    s, a, lens_dev = net._inputs.put(s, a, true_len)   # on the copy stream (hostsync.InputStage)
    head = next(iter(net.heads.values()))
    # sampled head: its negatives' row gather joins the embedding-gather launch
    # (and, catch-up Adam, the step's target and negative rows are brought up to date first)
    net.trunk.neg_job = head.neg_job("main", s.shape[0], tgt=a) if hasattr(head, "neg_job") else None
    h = net.trunk.forward(s, true_len, slot="main", save=True, lens_dev=lens_dev)
    B = h.shape[0]
    mask = None
    if net.training and net.dropout_p > 0:
        mask = net.dropout_mask(B)
        hd = net._hd.get(B)
        if hd is None:
            net._hd = {B: torch.empty_like(h)}
            hd = net._hd[B]
        h_in = net.apply_mask(h, mask, hd)
    else:
        h_in = h
    # the GRU forward's bf16 K-planes of h (sampled head) unless dropout changed h
    loss, _ = head.forward_loss(h_in, a, slot="main", h_planes=net.trunk.h_planes if mask is None else None)
    if host is not None:
        host.capture(loss)
    adam6 = clock.next_args()
    net.trunk_tag = getattr(net, "trunk_tag", 0) + 1
    dh = net.dh_buffer(B)
    # the head's pass 2 (dW + Adam) runs on a side stream under the trunk
    # backward (which needs only dh) and the next step's trunk forward; the
    # head joins it on the next access of its parameters or workspace
    head.backward_step(h_in, a, dh, adam6, slot="main", overlap=True)
    if mask is not None:
        net.apply_mask(dh, mask, dh)
    net.trunk.backward(dh, slot="main")
    net.trunk.step(adam6, net.trunk_tag)
    return loss
