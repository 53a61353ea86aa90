# round-4 profiles after the q-gram records: the configs[2] legs (kernel trace + VALU/FETCH/WRITE passes)
bash tools/profile_r03.sh r04q ed_clustered ed_survey ed_alphabet > gpurun_out/r04q.log 2>&1 || { tail -20 gpurun_out/r04q.log; exit 1; }
tail -2 gpurun_out/r04q.log
