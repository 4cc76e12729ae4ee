"""Item tokenizer with the reference's interface (``recommenders/utils/
tokenizer.py``): ``stoi`` / ``itos``, optional ``<unk>`` (before ``<pad>``,
so ``<pad>`` is the last index), ``extend``, ``len``, JSON ``save_to_file`` /
``from_file`` / ``from_dict`` with the same {"stoi", "itos"} layout.  Host
bookkeeping only; the device path consumes it through a lookup table
(recommenders/hip/remap.py)."""
from __future__ import annotations

import json


class Tokenizer:
    def __init__(self, vocabulary, unknown=False, padding=True):
        self.stoi_ = {}
        for tok in vocabulary:
            self.stoi_[tok] = len(self.stoi_)
        self.unknown = bool(unknown)
        if unknown:
            self.unk_token = "<unk>"
            self.unk_idx = len(self.stoi_)
            self.stoi_[self.unk_token] = self.unk_idx
        if padding:
            self.pad_token = "<pad>"
            self.pad_idx = len(self.stoi_)
            self.stoi_[self.pad_token] = self.pad_idx
        self.itos_ = [None] * len(self.stoi_)
        for tok, i in self.stoi_.items():
            self.itos_[i] = tok

    def stoi(self, string):
        if self.unknown:
            return self.stoi_.get(string, self.stoi_[self.unk_token])
        return self.stoi_[string]

    def itos(self, index):
        return self.itos_[index]

    def extend(self, new_vocabulary):
        """Reference numbering kept: the i-th new string maps to len - 1 + i
        in ``stoi``; ``itos`` appends the new strings."""
        base = len(self.stoi_) - 1
        new = {tok: base + i for i, tok in enumerate(new_vocabulary)}
        self.stoi_.update(new)
        self.itos_.extend(sorted(new, key=new.get))

    def __len__(self):
        return len(self.itos_)

    def save_to_file(self, file_path):
        with open(file_path, "w") as f:
            json.dump({"stoi": self.stoi_, "itos": self.itos_}, f)

    @classmethod
    def from_dict(cls, tokenizer_dict):
        tok = cls([], padding=False)
        tok.stoi_ = dict(tokenizer_dict["stoi"])
        tok.itos_ = list(tokenizer_dict["itos"])
        if "<pad>" in tok.stoi_:
            tok.padding = True
            tok.pad_token = "<pad>"
            tok.pad_idx = tok.stoi_["<pad>"]
        tok.unknown = "<unk>" in tok.stoi_
        if tok.unknown:
            tok.unk_token = "<unk>"
            tok.unk_idx = tok.stoi_["<unk>"]
        return tok

    @classmethod
    def from_file(cls, file_path):
        with open(file_path) as f:
            return cls.from_dict(json.load(f))
