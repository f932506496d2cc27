set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
export TK_EMULATE_NOCOMM=1
BARGS="--emulate-ranks 8 --no-end-to-end" bash tools/gpu/ab_env.sh n8:X=1 n8skipR:TKHIP_TEST_SKIP=1 n8skipP:TKHIP_TEST_SKIP=2 n8skipRP:TKHIP_TEST_SKIP=3 && \
BARGS="--no-end-to-end" bash tools/gpu/ab_env.sh n1:X=1 n1skipRP:TKHIP_TEST_SKIP=3 && \
BARGS="--config C1 --no-end-to-end" bash tools/gpu/ab_env.sh c1:X=1 c1skipRP:TKHIP_TEST_SKIP=3
