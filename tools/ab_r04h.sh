set -o pipefail
TAG=r04h/ab REPS=2 bash tools/abtest.sh base v2 lib rec
