set -o pipefail
O=gpurun_out/r2_v44; mkdir -p $O
timeout -k 10 120 python -u scripts/frame_scan_phases.py > $O/frame_scan_phases.txt 2>&1 && cat $O/frame_scan_phases.txt &&
timeout -k 10 300 python -u bench/world_rehearsal.py --world 2 --steps 8 --warmup 2 > $O/rehearsal_w2_plain.json 2> $O/rw2.err && cat $O/rehearsal_w2_plain.json &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_w8 -o run -- python3 bench/world_rehearsal.py --world 8 --steps 16 --warmup 4 > $O/prof_w8.log 2>&1 && tail -3 $O/prof_w8.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_w1 -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof_w1.log 2>&1
