set -u
bash tools/gpu_mel.sh "${1:-x}" || exit 1
PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU;TA_BUSY_avr TA_TA_BUSY_sum" timeout -k 10 400 bash tools/pmc_cmd.sh mel logmel2048 tools/mel_bench.py 1
