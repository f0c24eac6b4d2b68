set -o pipefail
tools/replay_variants.sh base epl1 epl2 base epl1 epl2 && TREE=sars-like tools/replay_variants.sh base epl1 epl2
