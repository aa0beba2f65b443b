set -o pipefail
cd $GRAFT_REPO_ROOT && export HSA_ENABLE_IPC_MODE_LEGACY=0 && O=gpurun_out/f32at && mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --config resnet18_cifar --precision fp32 > $O/static_$i.log 2>&1 || exit 1
  echo "static $i $(grep -o '"value": [0-9.]*' $O/static_$i.log)"
  DLMPI_CONV_AUTOTUNE=2 timeout -k 10 300 python bench.py --config resnet18_cifar --precision fp32 > $O/tuned_$i.log 2>&1 || exit 1
  echo "tuned $i $(grep -o '"value": [0-9.]*' $O/tuned_$i.log)"
done
grep "autotune" $O/tuned_1.log | sort | uniq > $O/plans.txt; wc -l $O/plans.txt
