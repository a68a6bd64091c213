set -o pipefail
mkdir -p gpurun_out
for m in bench heat idle launch; do
  timeout -k 10 120 python -u tools/slowstart_probe.py $m 200 > gpurun_out/ss_$m.log 2>&1 || { echo "fail $m"; exit 1; }
  head -2 gpurun_out/ss_$m.log
done
