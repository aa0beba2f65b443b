#!/bin/bash
# Round-6 numerics at bench scale: the UNet-512 training-parity test, then training curves at the
# bench shapes (ResNet-50 224^2 bs 256, UNet 512^2 bs 16) native vs stock autocast / fp32 (+ a second
# autocast seed for the SGD-noise spread).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6_numerics; mkdir -p $O
[ -n "$NOTEST" ] || { MIOPEN_FIND_MODE=FAST timeout -k 10 700 python -u -m pytest -m gpu -q -x -s --timeout 600 --timeout-method thread tests/test_benchscale_gpu.py -k "training_matches" 2>&1 | tee $O/benchscale_training.log
rc=$?; tail -1 $O/benchscale_training.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error|native|torch " $O/benchscale_training.log | head -20; exit 1; fi
grep -E "^native|^torch " $O/benchscale_training.log; }
[ -n "$NOCLS" ] || { timeout -k 10 900 python -u benchmarks/convergence.py --task cls --arch resnet50 --size 224 --batch 256 --steps ${STEPS:-400} --lr ${LR:-0.01} --warmup_steps 100 --noise 1 --impls ${IMPLS:-native,autocast,fp32} --torch_seeds 1 > $O/cls_r50_224.jsonl 2> $O/cls_r50_224.err || { echo cls failed; tail -5 $O/cls_r50_224.err; exit 1; }
python -c "import json,sys; [print(d['impl'], d['seed'], d['loss'][-1], d.get('accuracy'), d['seconds']) for d in map(json.loads, open('$O/cls_r50_224.jsonl'))]"; }
[ -n "$NOSEG" ] && exit 0
timeout -k 10 900 python -u benchmarks/convergence.py --task seg --size 512 --batch 16 --steps ${STEPS:-300} --log_every 10 --impls native,autocast,fp32 --torch_seeds 1 > $O/seg_unet_512.jsonl 2> $O/seg_unet_512.err || { echo seg failed; tail -5 $O/seg_unet_512.err; exit 1; }
python -c "import json,sys; [print(d['impl'], d['seed'], d['loss'][-1], d.get('dice'), d['seconds']) for d in map(json.loads, open('$O/seg_unet_512.jsonl'))]"
exit 0
