set -u
cd $GRAFT_REPO_ROOT
run() { name=$1; shift; timeout -k 10 400 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/$name.log; exit 1; }; echo "== $name"; python3 tools/show_bench.py gpurun_out/$name.log | grep -E "value|nfa "; }
run e_full_noout --query5 "every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C or e4=D) -> not E for 5 sec" --select5 "select e1.timestamp as a having a < 0"
run e_full_out1 --query5 "every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C or e4=D) -> not E for 5 sec"
run e_nostart_noout --query5 "every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C or e4=D)" --select5 "select e1.timestamp as a having a < 0"
run e_ab25_noout --query5 "every e1=A -> e2=B[price>e1.price]<2:5>" --select5 "select e1.timestamp as a having a < 0"
