set -u
cd $GRAFT_REPO_ROOT
run() { name=$1; shift; timeout -k 10 400 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/$name.log; exit 1; }; echo "== $name"; python3 tools/show_bench.py gpurun_out/$name.log | grep -E "value|nfa "; }
run d_full --variant pattern_count_not5s
run d_nostart --query5 "every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C or e4=D)"
run d_ab25 --query5 "every e1=A -> e2=B[price>e1.price]<2:5>"
run d_ab --query5 "every e1=A -> e2=B[price>e1.price]"
run d_ab25nf --query5 "every e1=A -> e2=B<2:5>"
run d_lit
