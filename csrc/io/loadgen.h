// Native HTTP/1.1 load generator (BASELINE config 5 over real connections); see loadgen.cpp.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace lp {

struct LoadResult {
  std::vector<double> latency;   // seconds per request (-1: no complete response)
  std::vector<int32_t> status;   // HTTP status per request
  double t_start = 0, t_end = 0; // burst start / last response (monotonic seconds)
  int64_t completed = 0;
};

// One request per connection, all connections established before the burst; connection c sends
// msgs[idx[c]] (a complete HTTP request). Blocks until every response arrived or timeout_s passed.
// nthreads client threads, each with its own slice of the connections and epoll set (one thread
// sending ~1 GB of bodies over loopback was the bottleneck of the burst, not the server).
LoadResult http_burst(const std::string& host, int port, const std::vector<std::string>& msgs,
                      const std::vector<int32_t>& idx, double timeout_s, int nthreads = 8);

}  // namespace lp
