# First-GPU-operation costs in fresh processes (tools/probe/first_op.hip), each mode twice.
set -o pipefail
for m in A B C D E F A B C D; do timeout -k 5 60 tools/probe/first_op $m || exit 1; done
