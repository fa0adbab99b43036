for pg in 4096 1024 512 256; do RL_PROBE_GRID=$pg TAG=probe$pg bash scripts/bench_brief.sh | head -1; done
for pg in 4096 1024 512; do RL_PERM_GRID=$pg TAG=perm$pg bash scripts/bench_brief.sh | head -1; done
