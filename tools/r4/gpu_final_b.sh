# round 4 end: the measurement record (rocprofv3 stats of the bench command, per-kernel PMC passes)
set -o pipefail
export TMPDIR=/tmp
bash tools/r4/profile.sh || exit $?
echo PROFILE_OK
