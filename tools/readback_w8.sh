set -o pipefail
O=gpurun_out/r06/rbw8; mkdir -p $O
for i in 1 2; do
 for arm in dev rb hipm; do
  case $arm in dev) a=0; e="";; rb) a=1; e="";; tiny) a=1; e="RT_PROBE_COPY_BYTES=65536";; nocons) a=1; e="RT_PROBE_NO_CONSUMER=1";; hipm) a=1; e="RT_PROBE_HIPMALLOC=1";; esac
  env $e timeout -k 10 120 python3 -u tools/readback_probe.py $a world8 > $O/${arm}_$i.log 2>&1 || { tail $O/${arm}_$i.log; exit 1; }
  tail -1 $O/${arm}_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_frame'], 'maxissue', max(d['issue_ms']), 'wait', round(sum(d['wait_ms']),2))" $arm
 done
done
