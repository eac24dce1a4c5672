#!/bin/bash
# Results-parity evidence for the build's physics: PPO-SA at the reference's
# defaults (--num-envs 4095, T = 128, reference/batch + ppo…:48-118) for 1e8 env-steps, then the
# post-training evaluation of ppo…:380-461 (goal-only rewards, vs the zero and OU teams).  The
# untrained policy is evaluated first as the baseline.  Run on the GPU box:
#   gpurun -- 'bash tools/learning_curve.sh'   (outputs under gpurun_out/, copied to profiles/r02_*)
set -o pipefail
P=rsoccer-isaac-cleanrl_amd/ppo_continuous_action_isaacgym.py
timeout -k 10 300 python -u $P --env-id sa --num-updates 0 --evaluate --eval-matches 3000 --save-path gpurun_out/lc_untrained --exp-name untrained > gpurun_out/lc_untrained.log 2>&1 && \
timeout -k 10 900 python -u $P --env-id sa --total-timesteps 100000000 --evaluate --eval-matches 10000 --save-path gpurun_out/lc_sa --exp-name lc > gpurun_out/lc_sa.log 2>&1
