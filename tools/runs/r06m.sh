# round-end evidence on the current build: smoke, PMC passes, kernel stats, the default bench line, the other configs
set -o pipefail
TAG=r06m bash tools/round_end.sh > gpurun_out/r06m.log 2>&1 || { tail -20 gpurun_out/r06m.log; exit 1; }
