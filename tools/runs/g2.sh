set -o pipefail
mkdir -p gpurun_out/g2
tools/gpu_step.sh 200 gpurun_out/g2/abl.log python -u tools/sweep.py --paths 0 --ablate 0,1,2 --lanes 4,8 --wgs 0 --steps 100 || exit 1
tools/gpu_step.sh 600 gpurun_out/g2/mix.log bash tools/pmc_mix.sh gpurun_out/g2/pmc --path 0 --lanes 8 --reps 5 || exit 1
python3 tools/pmc_summary.py gpurun_out/g2/pmc crc32 > gpurun_out/g2/pmc_summary.txt
python3 tools/pmc_summary.py gpurun_out/g2/pmc probe >> gpurun_out/g2/pmc_summary.txt
