set -o pipefail
mkdir -p gpurun_out/copy
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for m in d2h default nocu; do
  timeout -k 10 60 $R/tools/copy_probe $m > $R/gpurun_out/copy/$m.txt 2>&1 || exit 1
  timeout -k 10 90 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/copy/prof_$m -o run -- $R/tools/copy_probe $m > $R/gpurun_out/copy/prof_$m.log 2>&1 || exit 1
done
cat $R/gpurun_out/copy/*.txt
