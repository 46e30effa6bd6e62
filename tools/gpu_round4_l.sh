# round-4: rocprofv3 evidence at the bench's default step count, then the Winning-PoSt window-size sweep
bash tools/prof_round.sh r04b && echo "prof ok" && bash tools/winning_c_sweep.sh
