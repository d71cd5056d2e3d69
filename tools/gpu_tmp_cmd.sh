bash tools/gpu_evidence.sh r03b && bash tools/gpu_timeline.sh r03b
