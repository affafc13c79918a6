set -e
bash tools/gpu/experiments/r2_msm20.sh
bash tools/gpu/experiments/r2_tasks2.sh
