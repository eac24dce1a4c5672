#!/usr/bin/env bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit; the script stops at the first abnormal exit
# (fault / abort / segfault / timeout), and only continues past ordinary test failures.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r01}

run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "abnormal exit ($rc) in $name: stopping" | tee -a "$OUT/session.log"
    exit $rc
  fi
  return 0
}

STEPS=${STEPS:-tests,smoke,bench,prof}
case ",$STEPS," in *,tests,*) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;; esac
case ",$STEPS," in *,tplay,*) run pytest_play 600 python -m pytest tests/test_play.py -m gpu -x -q ;; esac
case ",$STEPS," in *,smoke,*) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;; esac
case ",$STEPS," in *,bench,*) run bench 400 python bench.py; run bench_eager 300 python bench.py --graph 0 --no-cpu-baseline ;; esac
case ",$STEPS," in *,benchsa,*) run bench_sa 300 python bench.py --mode sa --no-cpu-baseline ;; esac
case ",$STEPS," in *,prof,*)
  run rocprof_stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
      python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --l3-check-fields 0 ;;
esac
case ",$STEPS," in *,pmc,*)
  run rocprof_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$TAG" -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --l3-check-fields 0 --rollout-k 0
  run rocprof_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$TAG" -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --l3-check-fields 0 --rollout-k 0 ;;
esac
# the same two passes at 131,072 fields (406 MB per launch, past the 256 MiB Infinity Cache)
case ",$STEPS," in *,pmcl3,*)
  run rocprof_fetch_l3 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_l3_$TAG" -o run -- \
      python3 bench.py --fields 131072 --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --l3-check-fields 0 --rollout-k 0
  run rocprof_write_l3 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_l3_$TAG" -o run -- \
      python3 bench.py --fields 131072 --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --l3-check-fields 0 --rollout-k 0 ;;
esac
case ",$STEPS," in *,tupd,*) run pytest_update 600 python -u -m pytest tests/test_update.py tests/test_ppo.py tests/test_policy.py -m gpu -x -v --timeout 200 --timeout-method thread ;; esac
# the update's fused-epilogue GEMMs: unit tests, kernel bench vs torch, PPO update fused vs split
case ",$STEPS," in *,gemm,*)
  run pytest_update 500 python -u -m pytest tests/test_update.py -m gpu -x -v --timeout 120 --timeout-method thread
  run gemm_fused 300 python -u tools/gemm_fused_bench.py
  VSS_UPDATE_MLP=fused run ppo_fused 300 python -u rsoccer-isaac-cleanrl_amd/ppo_continuous_action_isaacgym.py --env-id sa --num-envs 65536 --num-updates 3 --log false
  # (needs tools/ab_switches_r04.patch applied: the split path is retired from the product)
  VSS_UPDATE_MLP=split run ppo_split 300 python -u rsoccer-isaac-cleanrl_amd/ppo_continuous_action_isaacgym.py --env-id sa --num-envs 65536 --num-updates 3 --log false ;;
esac
case ",$STEPS," in *,sa1e8,*)
  run ppo_sa_1e8 600 python -u rsoccer-isaac-cleanrl_amd/ppo_continuous_action_isaacgym.py --env-id sa --num-envs 65536 \
      --total-timesteps 100663296 --save-path "$OUT/runs_$TAG" ;;
esac
case ",$STEPS," in *,tdist,*) run pytest_dist 600 python -m pytest tests/test_dist.py -m gpu -x -q ;; esac
case ",$STEPS," in *,amp,*) run ppo_amp 900 python rsoccer-isaac-cleanrl_amd/ppo_continuous_action_isaacgym.py --env-id sa --num-envs 65536 --num-updates 2 --amp bf16 --save-path /tmp/runs ;; esac
case ",$STEPS," in *,ppoprof,*)
  run rocprof_ppo 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_ppo_$TAG" -o run -- \
      python3 rsoccer-isaac-cleanrl_amd/ppo_continuous_action_isaacgym.py --env-id sa --num-envs 65536 --num-updates 1 --log false ;;
esac
case ",$STEPS," in *,ppo,*) run ppo_sa 900 python rsoccer-isaac-cleanrl_amd/ppo_continuous_action_isaacgym.py --env-id sa --num-envs 65536 --num-updates 2 --save-path /tmp/runs ;; esac
# the full SA run to >= 1e8 env-steps (12 updates of 65,536 x 128), with its
# loss curves; config 4: DMA at 65,536 fields (196,608 agent rows), a short run + the step bench
case ",$STEPS," in *,ppo1e8,*)
  run ppo_sa_1e8 900 python rsoccer-isaac-cleanrl_amd/ppo_continuous_action_isaacgym.py --env-id sa --num-envs 65536 \
      --total-timesteps 100663296 --save-path "$OUT/runs_$TAG" && \
  run ppo_dma 900 python rsoccer-isaac-cleanrl_amd/ppo_continuous_action_isaacgym.py --env-id dma --num-envs 196608 \
      --num-updates 2 --save-path "$OUT/runs_$TAG" && \
  run bench_dma 300 python bench.py --mode dma --no-cpu-baseline --ppo-updates 0 ;; esac
case ",$STEPS," in *,sq,*)
  run rocprof_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d "$OUT/pmc_sq_$TAG" -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
  run rocprof_sq2 400 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq2_$TAG" -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
esac
case ",$STEPS," in *,profall,*)
  run prof_full 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
      python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --ppo-updates 0 --rollout-k 16
  run prof_sa 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_sa_$TAG" -o run -- \
      python3 bench.py --mode sa --steps 100 --warmup 10 --no-cpu-baseline --ppo-updates 0
  run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$TAG" -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --rollout-k 0
  run pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$TAG" -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --rollout-k 0
  run pmc_fetch_sa 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_sa_$TAG" -o run -- \
      python3 bench.py --mode sa --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0
  run pmc_write_sa 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_sa_$TAG" -o run -- \
      python3 bench.py --mode sa --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0
  run prof_policy 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_policy_$TAG" -o run -- \
      python3 tools/policy_bench.py
  run pmc_policy 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc_policy_$TAG" -o run -- \
      python3 tools/policy_bench.py ;;
esac
# the rollout policy kernel: parity tests, timing, MFMA-busy and stall counters (separate passes)
case ",$STEPS," in *,pol,*)
  run pytest_policy 300 python -u -m pytest tests/test_policy.py -m gpu -x -v --timeout 120 --timeout-method thread && \
  run policy_bench 300 python -u tools/policy_bench.py && \
  run pmc_policy 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc_policy_$TAG" -o run -- \
      python3 tools/policy_bench.py && \
  run pmc_policy_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU --output-format csv -d "$OUT/pmc_policy_sq_$TAG" -o run -- \
      python3 tools/policy_bench.py ;;
esac
# wall-clock to a trained policy (score >= 0.9 vs the zero team) at the reference's defaults
case ",$STEPS," in *,tts,*)
  run tts_sa_4095 900 python -u tools/time_to_score.py --env-id sa --num-envs 4095 --eval-every 10 --max-steps 3e8 ;; esac
case ",$STEPS," in *,tts65k,*)
  run tts_sa_65536 1100 python -u tools/time_to_score.py --env-id sa --num-envs 65536 --eval-every 8 --max-steps 1.6e9 ;; esac
echo "session done" | tee -a "$OUT/session.log"
