set -u -o pipefail
cd "$(dirname "$0")/.."
r() { timeout -k 10 200 python -u tools/dbg_cfg4.py "$@" || exit 1; }
IDF_LANES=2 r resflows_smallpatch_split 2 f32
IDF_LANES=2 IDF_LANE_STAGGER=none r resflows_smallpatch_split 2
IDF_LANES=2 r resflows_smallpatch_split 3
IDF_LANES=2 r resflows_smallpatch_split 4
IDF_LANES=3 r resflows_smallpatch_split 3
IDF_LANES=2 r resflow-patches-vqvae 32
IDF_LANES=2 r resflow-patches-vqvae 4
