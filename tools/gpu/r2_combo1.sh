set -e
bash tools/gpu/r2_msm20.sh
bash tools/gpu/r2_tasks2.sh
