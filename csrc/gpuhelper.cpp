// nos-gpuhelper: the partition agent's short-lived GPU helper as a native executable.
//
//   nos-gpuhelper barrier --votes 1,1,0,... [--expect N] [--backend xgmi|rccl]
//
// ``xgmi`` (default): a ring of peer-to-peer token writes over xGMI (csrc/p2p_barrier.hip), planned
// over the peer-capable links (csrc/ring_plan.h; a device without a peer path writes locally) —
// every device executes, every link of the ring carries its token; ``rccl``: one ncclCommInitAll
// clique and a grouped 4-byte all-reduce (csrc/rccl_barrier.cpp).
//
// The agent never initialises HIP itself (a KFD context in the agent would make every later mode
// switch fail with "busy"), so each node-atomic commit runs in a child process spawned after the
// flips. The Python helper (walkai_nos_amd/cmd/gpuhelper.py) spent 0.7 s starting an interpreter
// and importing before it touched the GPU and 2.0-6.0 s in hipInit + ncclCommInitAll
// (profiles/operator_gpu_report_r2.json); this executable starts in milliseconds and reports where
// the rest goes, phase by phase:
//
// Either way it prints ONE JSON line: n (votes), seen (HIP devices), sum, and the wall milliseconds of
// hip_init (hipInit + device count), comm_init (ncclCommInitAll over every device), allreduce (one
// grouped 4-byte sum), destroy, total. A device count different from --expect (or from the number
// of votes) is a veto: a partition that did not come up after the flip. RCCL init tunables that
// cost nothing for a 4-byte all-reduce (one channel, small buffers, no MSCCL) are applied unless
// the caller set them already (NOS_BARRIER_KEEP_NCCL_ENV=1 keeps RCCL's defaults).
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
const char* nos_barrier_last_error();
int nos_barrier_init_all(int ndev, const int* devlist, void** handle);
int nos_barrier_allreduce_all(void* handle, const int32_t* votes, int32_t* result);
int nos_barrier_destroy_all(void* handle);
const char* nos_p2p_last_error();
const char* nos_p2p_last_plan();
int nos_p2p_last_peer_links();
int nos_p2p_last_local();
int nos_p2p_barrier(int n, const int32_t* votes, int32_t* sum, int32_t* intact);
}

namespace {
using Clock = std::chrono::steady_clock;

double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += c;
    } else if (static_cast<unsigned char>(c) < 0x20) {
      o += ' ';
    } else {
      o += c;
    }
  }
  return o;
}

void tune_rccl_env() {
  if (const char* keep = std::getenv("NOS_BARRIER_KEEP_NCCL_ENV"); keep && std::strcmp(keep, "1") == 0) return;
  // a 4-byte all-reduce needs one channel and tiny buffers; every extra channel costs buffer
  // allocations and proxy setup per peer at init time
  const char* kv[][2] = {{"NCCL_MIN_NCHANNELS", "1"}, {"NCCL_MAX_NCHANNELS", "1"},
                         {"NCCL_BUFFSIZE", "65536"}, {"RCCL_MSCCL_ENABLE", "0"},
                         {"RCCL_MSCCLPP_ENABLE", "0"}, {"NCCL_IB_DISABLE", "1"},
                         {"NCCL_PROTO", "LL"}};
  for (auto& p : kv) setenv(p[0], p[1], /*overwrite=*/0);
}

int barrier(const std::vector<int32_t>& votes, int expect, const std::string& backend) {
  auto t0 = Clock::now();
  tune_rccl_env();
  std::string err;
  double hip_init = 0, comm_init = 0, allreduce = 0, destroy = 0;
  std::string ring;
  int peer_links = -1, local = -1;
  int seen = -1;
  int32_t sum = 0;
  hipError_t e = hipInit(0);
  if (e == hipSuccess) e = hipGetDeviceCount(&seen);
  hip_init = ms_since(t0);
  const int want = expect >= 0 ? expect : int(votes.size());
  if (e != hipSuccess) {
    err = std::string("hipInit/hipGetDeviceCount: ") + hipGetErrorString(e);
    seen = -1;
  } else if (seen != want || seen != int(votes.size())) {
    err = "helper sees " + std::to_string(seen) + " HIP devices, the device map has " + std::to_string(want) +
          " (" + std::to_string(votes.size()) + " votes)";
  } else if (backend == "xgmi") {
    auto t1 = Clock::now();
    int32_t intact = 0;
    int rc = nos_p2p_barrier(seen, votes.data(), &sum, &intact);
    comm_init = 0;
    allreduce = ms_since(t1);
    ring = nos_p2p_last_plan();
    peer_links = nos_p2p_last_peer_links();
    local = nos_p2p_last_local();
    if (rc == -3) {
      // a device did not complete its write before the deadline: report the veto and leave at once
      // (tearing the context down would wait for that device)
      std::printf("{\"n\": %zu, \"seen\": %d, \"sum\": 0, \"hip_init_ms\": %.3f, \"allreduce_ms\": %.3f, "
                  "\"total_ms\": %.3f, \"native\": true, \"backend\": \"xgmi\", \"error\": \"%s\"}\n",
                  votes.size(), seen, hip_init, allreduce, ms_since(t0), json_escape(nos_p2p_last_error()).c_str());
      std::fflush(stdout);
      std::_Exit(0);
    }
    if (rc != 0)
      err = std::string("p2p ring: ") + nos_p2p_last_error();
    else if (intact != seen)
      err = std::to_string(seen - intact) + " token(s) did not arrive intact over the ring";
  } else {
    std::vector<int> devs(seen);
    for (int i = 0; i < seen; ++i) devs[i] = i;
    void* h = nullptr;
    auto t1 = Clock::now();
    int rc = nos_barrier_init_all(seen, devs.data(), &h);
    comm_init = ms_since(t1);
    if (rc != 0) {
      err = std::string("init: ") + nos_barrier_last_error();
    } else {
      auto t2 = Clock::now();
      int32_t res = 0;
      rc = nos_barrier_allreduce_all(h, votes.data(), &res);
      allreduce = ms_since(t2);
      if (rc != 0)
        err = std::string("allreduce: ") + nos_barrier_last_error();
      else
        sum = res;
      auto t3 = Clock::now();
      if (nos_barrier_destroy_all(h) != 0 && err.empty()) err = std::string("destroy: ") + nos_barrier_last_error();
      destroy = ms_since(t3);
    }
  }
  std::printf("{\"n\": %zu, \"seen\": %d, \"sum\": %d, \"hip_init_ms\": %.3f, \"comm_init_ms\": %.3f, "
              "\"allreduce_ms\": %.3f, \"destroy_ms\": %.3f, \"total_ms\": %.3f, \"native\": true, "
              "\"backend\": \"%s\"",
              votes.size(), seen, err.empty() ? sum : 0, hip_init, comm_init, allreduce, destroy, ms_since(t0),
              backend.c_str());
  if (peer_links >= 0)
    std::printf(", \"ring\": \"%s\", \"peer_links\": %d, \"local_writes\": %d", json_escape(ring).c_str(),
                peer_links, local);
  if (!err.empty()) std::printf(", \"error\": \"%s\"", json_escape(err).c_str());
  std::printf("}\n");
  std::fflush(stdout);
  return 0;
}

int usage() {
  std::fprintf(stderr, "usage: nos-gpuhelper barrier --votes 1,1,0 [--expect N] [--backend xgmi|rccl]\n");
  return 2;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return usage();
  std::string cmd = argv[1];
  if (cmd != "barrier") return usage();
  std::vector<int32_t> votes;
  int expect = -1;
  std::string backend = "xgmi";
  for (int i = 2; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--votes" && i + 1 < argc) {
      std::string v = argv[++i];
      size_t pos = 0;
      while (pos < v.size()) {
        size_t c = v.find(',', pos);
        std::string tok = v.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
        if (!tok.empty()) votes.push_back(std::atoi(tok.c_str()) ? 1 : 0);
        if (c == std::string::npos) break;
        pos = c + 1;
      }
    } else if (a == "--expect" && i + 1 < argc) {
      expect = std::atoi(argv[++i]);
    } else if (a == "--backend" && i + 1 < argc) {
      backend = argv[++i];
      if (backend != "xgmi" && backend != "rccl") return usage();
    } else {
      return usage();
    }
  }
  if (votes.empty()) return usage();
  return barrier(votes, expect, backend);
}
