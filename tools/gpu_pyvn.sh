set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pyvn; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/py -o run --output-format csv -- python bench.py --steps 20 --warmup 5 > $O/py.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/nat -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 20 --warmup 3 > $O/nat.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/py_plain.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --graph > $O/py_graph.log 2>&1 || exit 1
timeout -k 10 200 build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 30 --warmup 3 > $O/nat_plain.log 2>&1 || exit 1
