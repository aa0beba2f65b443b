R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/prev_prof
for i in 1 2 3; do
  for t in new old; do
    d=$R; [ $t = old ] && d=$R/abprev
    (cd $d && timeout -k 10 300 python bench.py --config resnet18_cifar --steps 50 --warmup 5) > gpurun_out/prev_prof/c_${t}_$i.log 2>&1 || { echo "fail $t"; exit 1; }
    echo "$t #$i $(grep -o '"value": [0-9.]*' gpurun_out/prev_prof/c_${t}_$i.log)"
  done
done
for t in new old; do
  d=$R; [ $t = old ] && d=$R/abprev
  (cd $d && timeout -k 10 300 python -m cProfile -s tottime bench.py --config resnet18_cifar --steps 100 --warmup 5) > gpurun_out/prev_prof/prof_${t}.txt 2>&1 || { echo "prof fail $t"; exit 1; }
done
