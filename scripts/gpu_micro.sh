# Micro-benchmarks of data-plane primitives under a kernel trace (bench/micro/).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r3_micro}; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/t -o run -- ./bench/micro/sort_fence > $O/sort_fence.log 2>&1 || { tail -20 $O/sort_fence.log; exit 1; }
grep -v "^W\|^E" $O/sort_fence.log | tail -8
python3 bench/micro/parse_trace.py $O/t 50 | tee $O/sort_fence_trace.txt
rm -rf $O/t
