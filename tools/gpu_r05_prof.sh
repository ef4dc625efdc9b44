# Round-5 closing records, part 2: the headline kernel's trace stats with FETCH_SIZE / WRITE_SIZE passes, the
# per-kernel passes over tools/pmc_configs.py (trace stats, FETCH_SIZE, WRITE_SIZE), and the phase breakdown
# of one small request from host memory (S1 1 MiB, C1 4 MiB through rdx_execute_owned, one thread).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05p}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2trace -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --primary-only > $OUT/c2trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --primary-only > $OUT/pmc.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --primary-only > $OUT/pmcw.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/cfgtrace -o run --output-format csv -- python3 tools/pmc_configs.py 20 > $OUT/cfgtrace.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/cfg_fetch -o run --output-format csv -- python3 tools/pmc_configs.py 10 > $OUT/cfg_fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/cfg_write -o run --output-format csv -- python3 tools/pmc_configs.py 10 > $OUT/cfg_write.log 2>&1 &&
RDX_PHASES=1 timeout -k 10 60 $B s1 1 2000 owned >> $OUT/phases_conc.jsonl 2>> $OUT/phases_s1.jsonl &&
RDX_PHASES=1 timeout -k 10 60 $B c1 1 2000 owned >> $OUT/phases_conc.jsonl 2>> $OUT/phases_c1.jsonl &&
timeout -k 10 60 $B s1 1 2000 owned >> $OUT/phases_conc.jsonl &&
timeout -k 10 60 $B c1 1 2000 owned >> $OUT/phases_conc.jsonl &&
RDX_PINF_PROF=1 timeout -k 10 120 python3 tools/probe_pinflate.py 2 > $OUT/pinf_prof_probe.jsonl 2> $OUT/pinf_prof.txt
rc=$?
exit $rc
