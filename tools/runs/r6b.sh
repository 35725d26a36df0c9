set -o pipefail
# round 6 (b): the receive slots' own staging and the unlocked socket wait: the GPU
# suite (new: send while a receive waits, page-end arenas, a DGRAM ending on the arena), then
# the three traffic passes of this build (profiles/traffic_*.json now name their library)
out=gpurun_out/r6b
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest_harness.log python -u -m pytest tests/test_gpu_harness.py -m gpu -v --timeout 120 --timeout-method thread || exit 1
tools/gpu_step.sh 900 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
bash tools/traffic_passes.sh $out || exit 1
sha256sum enet-csharp_amd/libenethip.so > $out/lib_sha.txt
echo done > $out/done
