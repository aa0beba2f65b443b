R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/prev_ab
for i in 1 2; do
  for t in new old; do
    d=$R; [ $t = old ] && d=$R/abprev
    for c in resnet18_cifar resnet50; do
      (cd $d && timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5) > gpurun_out/prev_ab/${c}_${t}_$i.log 2>&1 || { echo "fail $t $c"; exit 1; }
      echo "$c $t #$i $(grep -o '"value": [0-9.]*' gpurun_out/prev_ab/${c}_${t}_$i.log)"
    done
  done
done
