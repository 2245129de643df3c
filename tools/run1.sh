set -o pipefail
bash tools/hp_piece.sh || exit 1
TAG=ab1 REPS=3 bash tools/abtest.sh lib bufw
