# round-4 profiles at HEAD: K1 and the two configs[2] legs (kernel trace + VALU/FETCH/WRITE counter passes)
bash tools/profile_r03.sh r04p replayable ed_clustered ed_survey ed_wide > gpurun_out/r04p.log 2>&1 || { tail -20 gpurun_out/r04p.log; exit 1; }
tail -3 gpurun_out/r04p.log
for l in replayable ed_clustered ed_survey ed_wide; do echo == $l; head -30 gpurun_out/r04p/$l/summary.txt; done
