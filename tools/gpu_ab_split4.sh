#!/bin/bash
# Heavy-row split parameters (engine.split_rows : engine.pieces) on the full
# config3 launch, in-tree library, two rounds.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-split4}
mkdir -p $O
export AB_CASES=16384:1 AB_REPS=3 AB_OPT=0
for round in 1 2; do
  for sp in ${SPLITS:-256:16 128:16 512:16 256:8 256:32 1024:8}; do
    AB_SPLIT=$sp timeout -k 10 300 python -u tools/ab_w.py > $O/split_${sp/:/_}_$round.log 2>&1 \
      || { echo "split $sp failed"; tail -20 $O/split_${sp/:/_}_$round.log; exit 1; }
    echo "split $sp #$round: $(grep digest $O/split_${sp/:/_}_$round.log | cut -c1-90)"
  done
done
