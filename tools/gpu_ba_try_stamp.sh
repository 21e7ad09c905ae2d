bash tools/gpu_ba_try.sh && bash tools/gpu_ba_stamp.sh && tail -3 gpurun_out/bastamp/stamps--hd.txt && tail -2 gpurun_out/bastamp/stamps.txt
