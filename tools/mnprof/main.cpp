// gprof driver for the host MultiNode path: the bench loop of hbnode_bench.cpp
// linked statically with hbnode.cpp (built -pg by tools/mnprof/build.sh), so
// gprof sees the host functions.  ./mnprof G rounds flags threads
#include <cstdio>
#include <cstdlib>
#include <cstdint>
extern "C" int hbnb_run2(int device, uint32_t G, uint32_t n, uint32_t warmup, uint32_t rounds, uint32_t flags,
                         uint32_t threads, double* out);
int main(int argc, char** argv) {
  const uint32_t G = argc > 1 ? atoi(argv[1]) : 1000, rounds = argc > 2 ? atoi(argv[2]) : 200;
  const uint32_t flags = argc > 3 ? atoi(argv[3]) : 3, threads = argc > 4 ? atoi(argv[4]) : 1;
  double out[32] = {};
  const int rc = hbnb_run2(0, G, 3, 2, rounds, flags, threads, out);
  std::printf("rc %d G %u rounds %u: %.4g s, %.0f acks -> %.4g MsgAppResp/s\n", rc, G, rounds, out[0], out[1],
              out[1] / out[0]);
  return rc;
}
