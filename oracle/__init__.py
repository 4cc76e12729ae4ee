"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

This package is the parity checker for the MI355X path, never the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product path
(``ikea-recommender-system_amd/recommenders``) must never import it; with
the HIP extension missing the product fails loudly instead of falling back.

It restates the reference's per-step training math on PyTorch-CPU with the
same third-party ops the reference uses (``nn.Embedding`` gather,
``pack_padded_sequence`` + ``nn.GRU``, ``nn.Linear``, ``CrossEntropyLoss``,
``torch.optim.Adam``), written functionally so every step of the reference
quirk list in SURVEY.md §0 is explicit.  Each function cites the reference
file:line it follows.

Pinning: ``tests/test_oracle_golden.py`` checks this restatement against
golden vectors produced by running the reference itself in the build
container (``tests/golden/make_golden.py``), plus the reference's own
known-answer tests (Q-helpers, HR/NDCG, novelty, preprocessing).
Extensions with no reference counterpart (sampled softmax, SMORL's third
reward, multi-GPU sharding) are marked "parity unpinned" where defined.
"""
