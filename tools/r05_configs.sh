#!/bin/bash
# round 5: the other BASELINE config shapes on one MI355X at the final head
O=gpurun_out/$1; mkdir -p $O
# configs[0] shape: arxiv-like RMAT (scale 17, ef 9), fan-out [10,10], d = 128
timeout -k 10 300 python bench.py --scale 17 --ef 9 --dim 128 --fan-out 10,10 --secondary none \
  > $O/bench_arxiv.json 2> $O/bench_arxiv.err || { tail -5 $O/bench_arxiv.err; exit 1; }
cut -c1-160 $O/bench_arxiv.json
# configs[1] at B = 8192 (saturation)
timeout -k 10 300 python bench.py --batch 8192 --secondary none --no-cpu-baseline \
  > $O/bench_b8192.json 2> $O/bench_b8192.err || { tail -5 $O/bench_b8192.err; exit 1; }
cut -c1-160 $O/bench_b8192.json
# configs[3]'s graph with the uniform sampler
timeout -k 10 600 python bench.py --scale 27 --ef 12 --dim 128 --secondary none --no-cpu-baseline \
  > $O/bench_papers.json 2> $O/bench_papers.err || { tail -5 $O/bench_papers.err; exit 1; }
cut -c1-160 $O/bench_papers.json
# configs[4] shape: RMAT-1B (scale 26, ef 16), d = 256, one GPU
timeout -k 10 900 python bench.py --scale 26 --ef 16 --dim 256 --secondary none --no-cpu-baseline \
  > $O/bench_rmat1b.json 2> $O/bench_rmat1b.err || { tail -5 $O/bench_rmat1b.err; exit 1; }
cut -c1-160 $O/bench_rmat1b.json
