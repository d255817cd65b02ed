set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/sk; mkdir -p $O
for r in 1 2; do
  MVS_LIB=$PWD/ab/libmvs_A.so timeout -k 10 120 python3 scripts/bench_kernels.py cvt slic boundary sweep_spixl > $O/A$r.json 2>$O/A.err || { tail -5 $O/A.err; exit 1; }
  timeout -k 10 120 python3 scripts/bench_kernels.py cvt slic boundary sweep_spixl > $O/B$r.json 2>$O/B.err || { tail -5 $O/B.err; exit 1; }
  echo "A $(cat $O/A$r.json)"; echo "B $(cat $O/B$r.json)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr -o run -- python3 scripts/bench_kernels.py slic > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 scripts/kstats.py $O/tr
MVS_LIB=$PWD/ab/libmvs_A.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trA -o run -- python3 scripts/bench_kernels.py slic > $O/trA.log 2>&1 || { tail -5 $O/trA.log; exit 1; }
python3 scripts/kstats.py $O/trA
