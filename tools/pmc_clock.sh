set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_clk
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_clk/pass1 -o p -- python3 tools/round_profile.py c4 1 > gpurun_out/pmc_clk/pass1.log 2>&1
