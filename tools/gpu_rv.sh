set -o pipefail
tools/replay_variants.sh base dfstm dfsne dfst8 base && TREE=sars-like tools/replay_variants.sh base dfst8
