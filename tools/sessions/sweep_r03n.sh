# round 3: channels per ring at 4 ranks (512 MiB RS / AG / AR), then the GPU suite
SWEEP_CH="8 10" SWEEP_SLICE="524288" bash tools/ring_geom_sweep.sh r03n 4 &&
bash tools/gpu_run.sh r03n test
