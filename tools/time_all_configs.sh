set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export FR_SCENE_JIT="${FR_SCENE_JIT:-1}"  # the scene-specialised kernel, as the bench runs it
T="timeout -k 10 120 python3 tools/time_config.py"
: > gpurun_out/configs.jsonl
$T scene_01 256 256 4 4 5 >> gpurun_out/configs.jsonl &&
$T scene_01 1920 1080 64 8 3 >> gpurun_out/configs.jsonl &&
$T scene_08 1920 1080 256 8 3 >> gpurun_out/configs.jsonl &&
$T scene_08 1920 1080 256 8 5 2 >> gpurun_out/configs.jsonl &&
$T scene_08 1920 1080 256 8 5 4 >> gpurun_out/configs.jsonl &&
$T scene_08 1920 1080 256 8 5 8 >> gpurun_out/configs.jsonl &&
$T scene_08 3840 2160 1024 8 3 8 >> gpurun_out/configs.jsonl &&
$T gen:10000:sphere 1920 1080 512 8 3 >> gpurun_out/configs.jsonl &&
$T scene_06 1920 1080 64 8 3 >> gpurun_out/configs.jsonl &&
$T scene_02 1920 1080 64 8 3 >> gpurun_out/configs.jsonl &&
$T scene_04 1920 1080 64 8 3 >> gpurun_out/configs.jsonl &&
$T scene_05 1920 1080 64 8 3 >> gpurun_out/configs.jsonl
