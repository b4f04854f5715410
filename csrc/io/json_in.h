// Native decoder of POST /parse request bodies (see json_in.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

namespace lp {

enum { JIN_OK = 0, JIN_INVALID = 1, JIN_NOT_OBJECT = 2, JIN_FALLBACK = 3 };

struct PodRequest {
  bool pod_nonnull = false;   // `pod` present and not null (Parse.java:45)
  bool has_name = false;      // pod.metadata.name is a string
  std::string pod_name;
  int logs_kind = 0;          // 0 absent / null, 1 string, 2 other type
  std::string logs;           // UTF-8, escapes decoded
};

int parse_pod_request(const uint8_t* body, size_t n, PodRequest& out);

}  // namespace lp
