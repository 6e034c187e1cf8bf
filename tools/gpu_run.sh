#!/bin/bash
# One GPU-box session (run through gpurun from the repo root):
#   tools/gpu_run.sh <label> <step> [<step> ...]
# steps: test      pytest -m gpu (one process, per-test timeout)
#        test:<k>  pytest -m gpu -k <k>
#        bench     bench.py at N=1 (the driver's default invocation)
#        prof      rocprofv3 --kernel-trace --stats of bench.py (no CPU leg)
#        n2        bench.py N>1 rehearsal: 2 ranks sharing the one GPU
#        nr:<n>    the same with n ranks
#        spawn:<n> bench.py --gpus <n> without torch.distributed.run (the
#                  script starts its own rank processes)
#        smoke     __graft_entry__.smoke()
#        py:<file> python <file> (a tool script)
#        sweep:<mode>  tools/sweep_rc.py with SWEEP_MODE=<mode> (6 rounds)
#        pmcshapes tools/pmc_shapes.py (PMC passes over 2->2, copy, 2->1 shapes)
#        pmc       tools/pmc_traffic.py (separate FETCH_SIZE / WRITE_SIZE passes)
#        lat:<n>   tools/coll_latency.py on n ranks sharing the GPU (LAT_* env)
#        mprof:<n> the N>1 bench line on n ranks sharing the GPU, every rank
#                  under rocprofv3 --kernel-trace --stats (tools/mp_prof.py)
#        fence:<n> tools/fence_cost.py on n ranks (fences off / on, interleaved)
#        lll:<n>[q<k>]  tools/ll_latency.py on n ranks, GPU_MAX_HW_QUEUES=k (4)
#        lltrace:<n> the same under rocprofv3 kernel + HIP API trace per rank, tools/ll_trace.py summary
#        ll1p:<n>  the LL all-reduce with n ranks in ONE process (tools/ll_latency_1proc.py)
#        net:<n>   tools/net_rate.py on n ranks (xGMI ring vs the net proxy path,
#                  staging copies included)
#        fuzz:<n>[s<seed>]  tools/fuzz_coll.py on n ranks (random calls, paths,
#                  groups; bit-exact; FUZZ_SECONDS 240, FUZZ_ITERS 400)
# Outputs go to gpurun_out/<label>/.  Every GPU step has its own time limit
# and the chain stops at the first failure (no retries).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$1; shift
O=$R/gpurun_out/$L; mkdir -p $O
cd $R
export TMPDIR=/tmp
for s in "$@"; do
  echo "== $s $(date +%T)"
  case $s in
    test) timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 ;;
    test:*) lg=$(printf %s "${s#test:}" | tr -c 'A-Za-z0-9_' '_'); timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${s#test:}" > "$O/pytest_$lg.log" 2>&1 ;;
    bench) timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err ;;
    prof) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-extras > $O/bench_prof.json 2> $O/bench_prof.err) ;;
    n2) timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err ;;
    nr:*) timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${s#nr:} --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus ${s#nr:} --steps 5 --warmup 2 > $O/bench_n${s#nr:}.json 2> $O/bench_n${s#nr:}.err ;;
    spawn:*) timeout -k 10 900 python bench.py --gpus ${s#spawn:} --steps 5 --warmup 2 > $O/bench_spawn_n${s#spawn:}.json 2> $O/bench_spawn_n${s#spawn:}.err ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    py:*) timeout -k 10 600 python -u ${s#py:} > $O/$(basename ${s#py:} .py).log 2>&1 ;;
    sweep:*) SWEEP_MODE=${s#sweep:} SWEEP_ROUNDS=${SWEEP_ROUNDS:-6} timeout -k 10 300 python -u tools/sweep_rc.py > $O/sweep_${s#sweep:}.log 2>&1 ;;
    pmcshapes) timeout -k 10 200 python -u tools/rc_shape_driver.py > $O/rc_shape_driver.log 2>&1 && timeout -k 10 500 python -u tools/pmc_shapes.py > $O/pmc_shapes.log 2>&1 && cp gpurun_out/pmc_shapes.json $O/ ;;
    pmc) timeout -k 10 400 python -u tools/pmc_traffic.py > $O/pmc_traffic.log 2>&1 && cp gpurun_out/pmc_traffic.json $O/ ;;
    lat:*) timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${s#lat:} --master-addr 127.0.0.1 --master-port 29534 tools/coll_latency.py > $O/lat_n${s#lat:}.log 2> $O/lat_n${s#lat:}.err ;;
    mprof:*) timeout -k 10 600 python -u tools/mp_prof.py ${s#mprof:} $O/mprof_n${s#mprof:} --steps 5 --warmup 2 > $O/mprof_n${s#mprof:}.log 2>&1 ;;
    fence:*) timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${s#fence:} --master-addr 127.0.0.1 --master-port 29536 tools/fence_cost.py > $O/fence_n${s#fence:}.json 2> $O/fence_n${s#fence:}.err ;;
    lll:*) n=${s#lll:}; q=${n#*q}; n=${n%q*}; [ "$q" = "$n" ] && q=4; GPU_MAX_HW_QUEUES=$q timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29537 tools/ll_latency.py > $O/lll_n${n}_q${q}.json 2> $O/lll_n${n}_q${q}.err ;;
    lltrace:*) n=${s#lltrace:}; MP_PROF_SCRIPT=tools/ll_latency.py MP_PROF_FLAGS=--hip-runtime-trace timeout -k 10 600 python -u tools/mp_prof.py $n $O/lltrace_n$n > $O/lltrace_n$n.log 2>&1 && python tools/ll_trace.py $O/lltrace_n$n > $O/lltrace_n$n.json ;;
    ll1p:*) VCCL_ALLOW_SHARED_DEVICE=1 timeout -k 10 300 python -u tools/ll_latency_1proc.py ${s#ll1p:} > $O/ll1p_n${s#ll1p:}.json 2> $O/ll1p_n${s#ll1p:}.err ;;
    net:*) timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${s#net:} --master-addr 127.0.0.1 --master-port 29539 tools/net_rate.py > $O/net_n${s#net:}.json 2> $O/net_n${s#net:}.err ;;
    fuzz:*) n=${s#fuzz:}; sd=1; case $n in *s*) sd=${n#*s}; n=${n%%s*};; esac; FUZZ_SEED=$sd FUZZ_ITERS=${FUZZ_ITERS:-400} FUZZ_SECONDS=${FUZZ_SECONDS:-240} timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29538 tools/fuzz_coll.py > $O/fuzz_n${n}_s${sd}.json 2> $O/fuzz_n${n}_s${sd}.err ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
