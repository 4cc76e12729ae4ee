#!/bin/bash
# round 4: r05f (bias-late sampled logits, suite) then r05g (C5 step-only profile)
bash tools/rounds/r05f.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/rounds/r05g.sh; rc2=$?
exit $(( rc > rc2 ? rc : rc2 ))
