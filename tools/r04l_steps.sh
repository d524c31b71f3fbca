set -u
bash tools/probe_ab.sh gpurun_out/r04l_probe l1_c2_dgrad16,l1_c3_dgrad16,l2_c2_dgrad16,l2_c3_dgrad16,l3_c2_dgrad16,l1_c1_dgrad16 lbt_amd/liblbt_dfxp.so lbt_amd/build_var/occ4/liblbt_dfxp.so || exit 1
bash tools/ab_bench.sh gpurun_out/r04l 2 lbt_amd/liblbt_dfxp.so lbt_amd/build_var/tailplain/liblbt_dfxp.so lbt_amd/build_var/proplain/liblbt_dfxp.so lbt_amd/build_var/bothplain/liblbt_dfxp.so
