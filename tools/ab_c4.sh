# A/B of a variant library against the default one on the C4 bench line,
# alternating A B A B (run from the repo root via gpurun):
#   VARIANT=lodestar_amd/libbgv_x.so bash tools/ab_c4.sh
# The variant is built here first, e.g.
#   python3 -c "import sys; sys.path.insert(0, 'tools'); import build; build.build(lib='lodestar_amd/libbgv_x.so', defines=('KNOB=1',))"
# Each GPU step has its own time limit and the steps are chained with &&.
VARIANT=${VARIANT:-lodestar_amd/libbgv_x.so}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
timeout -k 10 200 python3 bench.py --no-c2 --no-cpu --steps 10 > gpurun_out/ab/a1.json 2>gpurun_out/ab/a1.log &&
BGV_LIB=$VARIANT timeout -k 10 200 python3 bench.py --no-c2 --no-cpu --steps 10 > gpurun_out/ab/b1.json 2>gpurun_out/ab/b1.log &&
timeout -k 10 200 python3 bench.py --no-c2 --no-cpu --steps 10 > gpurun_out/ab/a2.json 2>gpurun_out/ab/a2.log &&
BGV_LIB=$VARIANT timeout -k 10 200 python3 bench.py --no-c2 --no-cpu --steps 10 > gpurun_out/ab/b2.json 2>gpurun_out/ab/b2.log &&
timeout -k 10 200 python3 bench.py --no-c2 --no-cpu --steps 10 > gpurun_out/ab/a3.json 2>gpurun_out/ab/a3.log &&
BGV_LIB=$VARIANT timeout -k 10 200 python3 bench.py --no-c2 --no-cpu --steps 10 > gpurun_out/ab/b3.json 2>gpurun_out/ab/b3.log
