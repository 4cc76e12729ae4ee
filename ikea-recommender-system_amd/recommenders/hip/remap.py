"""Device tokenizer remap: the reference maps predicted
ids from the output to the input vocabulary element by element on the CPU
(``tensor.apply_(lambda x: input_tokenizer.stoi(output_tokenizer.itos(x)))``,
diversity.py:55-60, repetitiveness.py:42-47).  Here the map is tabulated once
per tokenizer pair (lut[j] = stoi(itos(j)), -1 where the reference would
raise) and applied by a gather kernel (csrc/misc.hip rg_remap_ids)."""
from __future__ import annotations

import torch

from . import call, stream_ptr

_CACHE = {}


def host_table(input_tokenizer, output_tokenizer):
    """int32 host table lut[j] = stoi(itos(j)) over the output vocabulary (-1
    where the reference's stoi raises), built once per tokenizer pair."""
    key = (id(input_tokenizer), id(output_tokenizer), "host")
    hit = _CACHE.get(key)
    if hit is not None and hit[0] is input_tokenizer and hit[1] is output_tokenizer:
        return hit[2]
    lut = []
    for j in range(len(output_tokenizer)):
        try:
            lut.append(int(input_tokenizer.stoi(output_tokenizer.itos(j))))
        except (KeyError, IndexError):
            lut.append(-1)
    t = torch.tensor(lut, dtype=torch.int32)
    _CACHE[key] = (input_tokenizer, output_tokenizer, t)
    return t


def remap_table(input_tokenizer, output_tokenizer, device):
    """The host table on ``device``, cached per (pair, device)."""
    key = (id(input_tokenizer), id(output_tokenizer), str(device))
    hit = _CACHE.get(key)
    if hit is not None and hit[0] is input_tokenizer and hit[1] is output_tokenizer:
        return hit[2]
    t = host_table(input_tokenizer, output_tokenizer).to(device)
    _CACHE[key] = (input_tokenizer, output_tokenizer, t)
    return t


class RemapError(KeyError):
    pass


def raise_if_unmapped(err, comm=None):
    """Raise RemapError if a remapped id had no input-vocabulary token, where
    the reference's ``stoi`` raises KeyError inside the reward (diversity.py:
    55-60) — i.e. before its backward / optimizer step.  Called between the
    rewards and the first parameter update (one host sync, tokenizer runs
    only); on an item-sharded step the flag is summed over the ranks first so
    every rank raises together."""
    if comm is not None:
        comm.all_reduce(err)
    if int(err.item()):
        err.zero_()
        raise RemapError("a predicted id has no input-vocabulary token (input_tokenizer.stoi(output_tokenizer.itos(id)))")


def remap_ids(idx, lut, err=None):
    """int32 (…) ids -> input-vocabulary ids (same shape), on idx's stream."""
    out = torch.empty_like(idx)
    call("rg_remap_ids", idx.data_ptr(), idx.numel(), lut.data_ptr(), lut.numel(), out.data_ptr(),
         None if err is None else err.data_ptr(), stream_ptr())
    return out


def tokenizers(input_tokenizer, output_tokenizer):
    """Both or neither (the reference tests ``input_tokenizer != None`` and then uses both)."""
    if input_tokenizer is None:
        return False
    if output_tokenizer is None:
        raise ValueError("input_tokenizer given without output_tokenizer")
    return True
