# Evidence for every roofline fraction bench.py reports, one round tag:
#   profiles/<tag>_kstats_<corpus>_L<level>.csv   rocprofv3 --kernel-trace --stats of
#       tools/kernel_times.py 1024 <corpus> <level> (3 deflate + 3 inflate calls, 1 GiB)
#   profiles/<tag>_kstats_c3_zlib1.csv            the same for tools/foreign_probe.py (C3's
#       zlib level-1 stream of the 25,165,962-B bmp, path 5, 3 inflate calls)
#   profiles/traffic.json                         HBM bytes per launch from FETCH_SIZE (x2,
#       the gfx950 correction) + WRITE_SIZE passes of tools/deflate_once.py / foreign_probe.py
# usage: on the GPU box `bash tools/profile_all.sh run` (results under gpurun_out/prof_all,
# which gpurun merges back), then here `bash tools/profile_all.sh collect r03` (profiles/).
set -e
mode=${1:-run}
tag=${2:-r06}
P=gpurun_out/prof_all
SPECS=${SPECS:-"repeat:2 text:2 mixed:2 random:2 zeros:2 bmp:2 text:3"}
N=1073741824
export DMX_ROUND=$tag
if [ "$mode" = collect ]; then
  for spec in $SPECS; do
    c=${spec%%:*}; l=${spec#*:}
    [ -d $P/s_$c$l ] || continue
    # (the newest run's file: gpurun merges every box's results into the local gpurun_out/)
    cp $(ls -t $(find $P/s_$c$l -name "*kernel_stats.csv") | head -1) profiles/${tag}_kstats_${c}_L$l.csv
    for k in k_deflate_segments k_deflate_emit k_inflate_lanes k_inflate_pj_list; do
      python3 tools/traffic.py $P/f_$c$l $P/w_$c$l $c:$N:$l:$k $k profiles/traffic.json || true
    done
    # (templated names: the workgroup resolve and the one-wave resolve of long token lists, two
    # launches per call, each averaged over its own dispatches; not the 64 KiB half resolve)
    python3 tools/traffic.py $P/f_$c$l $P/w_$c$l $c:$N:$l:k_inflate_resolve "k_inflate_resolve<32768u, 256u>" profiles/traffic.json || true
    python3 tools/traffic.py $P/f_$c$l $P/w_$c$l $c:$N:$l:k_inflate_resolve_wave "k_inflate_resolve<32768u, 64u>" profiles/traffic.json || true
  done
  # config C4's 64 KiB blocks (bench sub-record c4_64k): the mixed corpus at segment_bytes 65536
  if [ -d $P/s_c4 ]; then
    cp $(ls -t $(find $P/s_c4 -name "*kernel_stats.csv") | head -1) profiles/${tag}_kstats_c4_64k_L2.csv
    for k in k_deflate_segments k_deflate_emit k_inflate_lanes; do
      python3 tools/traffic.py $P/f_c4 $P/w_c4 c4_64k:$N:2:$k $k profiles/traffic.json || true
    done
    python3 tools/traffic.py $P/f_c4 $P/w_c4 c4_64k:$N:2:k_inflate_resolve_half "k_inflate_resolve_half<256u>" profiles/traffic.json || true
    python3 tools/traffic.py $P/f_c4 $P/w_c4 c4_64k:$N:2:k_inflate_resolve_half_wave "k_inflate_resolve_half<64u>" profiles/traffic.json || true
    python3 tools/traffic.py $P/f_c4 $P/w_c4 c4_64k:$N:2:k_inflate_resolve "k_inflate_resolve<65536u, 256u>" profiles/traffic.json || true
    python3 tools/traffic.py $P/f_c4 $P/w_c4 c4_64k:$N:2:k_inflate_resolve_wave "k_inflate_resolve<65536u, 64u>" profiles/traffic.json || true
  fi
  if [ -d $P/s_c3 ]; then
    cp $(ls -t $(find $P/s_c3 -name "*kernel_stats.csv") | head -1) profiles/${tag}_kstats_c3_zlib1.csv
    for k in k_fb_scan k_fb_compact k_fb_check k_fb_pdecode k_fb_units k_fb_win_init k_fb_win_jump k_fb_final \
             k_marker_count k_marker_write k_scan_part k_scan_apply; do
      python3 tools/traffic.py $P/f_c3 $P/w_c3 c3_zlib1:$k $k profiles/traffic.json || true
    done
  fi
  exit 0
fi
mkdir -p $P && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for spec in $SPECS; do
  c=${spec%%:*}; l=${spec#*:}
  rm -rf $P/s_$c$l $P/f_$c$l $P/w_$c$l
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $P/s_$c$l --output-format csv -- python3 tools/kernel_times.py 1024 $c $l > $P/kt_$c$l.txt 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/f_$c$l --output-format csv -- python3 tools/deflate_once.py $c 1024 $l 1 > /dev/null 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/w_$c$l --output-format csv -- python3 tools/deflate_once.py $c 1024 $l 1 > /dev/null 2>&1
  echo "$spec done"
done
if [ "${C4:-1}" = 1 ]; then
  rm -rf $P/s_c4 $P/f_c4 $P/w_c4
  DMX_SEG=65536 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $P/s_c4 --output-format csv -- python3 tools/kernel_times.py 1024 mixed 2 > $P/kt_c4.txt 2>&1
  DMX_SEG=65536 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/f_c4 --output-format csv -- python3 tools/deflate_once.py mixed 1024 2 1 > /dev/null 2>&1
  DMX_SEG=65536 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/w_c4 --output-format csv -- python3 tools/deflate_once.py mixed 1024 2 1 > /dev/null 2>&1
  echo "c4 done"
fi
if [ "${C3:-1}" = 1 ]; then
  rm -rf $P/s_c3 $P/f_c3 $P/w_c3
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $P/s_c3 --output-format csv -- python3 tools/foreign_probe.py > $P/c3.txt 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/f_c3 --output-format csv -- python3 tools/foreign_probe.py > /dev/null 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/w_c3 --output-format csv -- python3 tools/foreign_probe.py > /dev/null 2>&1
  cat $P/c3.txt
fi
