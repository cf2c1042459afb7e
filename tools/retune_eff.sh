#!/bin/bash
# per-layer autotune of EfficientNet-B7 at b32 (project convs now LDS-DMA GEMMs with per-image weights)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 800 python -u bench.py --model efficientnet_b7 --steps 20 --warmup 5 --retune --save-tuning gpurun_out/eff_tune.json > gpurun_out/eff_retune.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --model efficientnet_b7 --steps 20 --warmup 5 --tuning gpurun_out/eff_tune.json > gpurun_out/eff_newtab.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --model efficientnet_b7 --steps 20 --warmup 5 > gpurun_out/eff_oldtab.log 2>&1 || exit $?
echo "retuned $(grep -o '"value": [0-9.]*' gpurun_out/eff_retune.log)  new table $(grep -o '"value": [0-9.]*' gpurun_out/eff_newtab.log)  old table $(grep -o '"value": [0-9.]*' gpurun_out/eff_oldtab.log)"
