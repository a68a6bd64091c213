cd /root/repo
for l in A B A B; do echo "lib $l"; TRLX_T5_AMD_LIB=$PWD/ab/lib_$l.so LM_VARIANTS=8 timeout -k 10 300 python3 tools/lmhead_bench.py 2>/dev/null | grep -E "C4|variants" | tail -2; done
