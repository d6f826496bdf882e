# A/B build for tools/bcube_threads_stress.py: tools/ab/libgloo_amd_coarse_inbox.so is
# the product library with round 5's rule for the inbox arena's grain (coarse-grained
# hipMalloc memory when the writing ranks share this GPU in this process), nothing else
# changed.  Measurement only; load it with GLOO_AMD_LIB.
set -e
cd "$(dirname "$0")/../gloo_amd"
make -s libgloo_amd.so
mkdir -p ../tools/ab/obj
sed 's/fineArena_ = !hostArena_ && !recvPeers.empty();/fineArena_ = !hostArena_ \&\& !recvPeers.empty() \&\& !sharesDeviceInProcess;/' \
  csrc/executor.cc > ../tools/ab/obj/executor_coarse.cc
grep -q 'recvPeers.empty() && !sharesDeviceInProcess;' ../tools/ab/obj/executor_coarse.cc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I../include -Iinclude -Icsrc \
  -c ../tools/ab/obj/executor_coarse.cc -o ../tools/ab/obj/executor_coarse.o
objs=$(ls build/*.o | grep -v '^build/executor\.cc\.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $objs ../tools/ab/obj/executor_coarse.o -o ../tools/ab/libgloo_amd_coarse_inbox.so
echo "built tools/ab/libgloo_amd_coarse_inbox.so"
