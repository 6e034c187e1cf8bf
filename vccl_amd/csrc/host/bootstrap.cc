// TCP rendezvous for communicator creation.
//
// Reference behaviour (src/bootstrap.cc:399-1037): ncclGetUniqueId opens a
// root socket and returns its address inside the 128-byte id; every rank
// connects to it in ncclCommInitRank; bootstrapAllGather / barrier follow.
// This implementation is a star instead of the reference's socket ring: the
// root thread (in the process that created the id) stays alive for the
// communicator's lifetime and answers each all-gather round; single-node rings
// need only a handful of rounds (init, teardown), so the star costs nothing.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <random>
#include <thread>

#include "../../../include/vccl_bootstrap.h"
#include "core.h"

namespace vccl {

namespace {
constexpr uint64_t kIdMagic = 0x5643434c49443031ull;   // "VCCLID01"
constexpr uint64_t kHelloMagic = 0x5643434c48454c4full; // "VCCLHELO"

struct IdLayout {
  uint64_t magic;
  uint64_t nonce;
  sockaddr_in addr;
};
static_assert(sizeof(IdLayout) <= NCCL_UNIQUE_ID_BYTES, "id too small");

struct Hello {
  uint64_t magic, nonce;
  int32_t rank, nranks;
};

bool send_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= (size_t)k;
  }
  return true;
}
bool recv_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= (size_t)k;
  }
  return true;
}

void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

// Root: accept nranks ranks, then serve all-gather rounds until all close.
void root_main(int lfd, uint64_t nonce) {
  std::vector<int> fds;
  int nranks = -1, joined = 0;
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::seconds(param_int("BOOTSTRAP_TIMEOUT", 600));
  while (nranks < 0 || joined < nranks) {
    pollfd pfd{lfd, POLLIN, 0};
    int pr = poll(&pfd, 1, 1000);
    if (std::chrono::steady_clock::now() > deadline) {
      VWARN("bootstrap root: timed out waiting for ranks (%d joined)", joined);
      goto done;
    }
    if (pr <= 0) continue;
    int fd = accept(lfd, nullptr, nullptr);
    if (fd < 0) continue;
    set_nodelay(fd);
    // A connection that never sends its Hello (a stale rank, a port probe)
    // must not stall the rendezvous: bounded read, then blocking again for
    // the all-gather rounds (which legitimately wait for the slowest rank).
    timeval tv{(time_t)param_int("BOOTSTRAP_HELLO_TIMEOUT_S", 10), 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    Hello h;
    const bool got = recv_all(fd, &h, sizeof(h));
    timeval none{0, 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof(none));
    if (!got || h.magic != kHelloMagic || h.nonce != nonce ||
        h.nranks <= 0 || h.rank < 0 || h.rank >= h.nranks || (nranks >= 0 && h.nranks != nranks)) {
      close(fd);
      continue;
    }
    if (nranks < 0) {
      nranks = h.nranks;
      fds.assign(nranks, -1);
    }
    if (fds[h.rank] != -1) {
      close(fd);
      continue;
    }
    fds[h.rank] = fd;
    joined++;
  }
  // all-gather rounds
  for (;;) {
    uint64_t len = 0;
    std::vector<char> all;
    bool ok = true;
    for (int r = 0; r < nranks && ok; r++) {
      uint64_t l;
      if (!recv_all(fds[r], &l, sizeof(l))) { ok = false; break; }
      if (r == 0) {
        len = l;
        all.resize(len * nranks);
      } else if (l != len) {
        ok = false;
        break;
      }
      if (len && !recv_all(fds[r], all.data() + r * len, len)) ok = false;
    }
    if (!ok) break;  // a rank closed: the communicator is gone
    for (int r = 0; r < nranks; r++) send_all(fds[r], all.data(), all.size());
  }
done:
  for (int fd : fds)
    if (fd >= 0) close(fd);
  close(lfd);
}
}  // namespace

struct Bootstrap {
  int fd = -1;
  int rank = 0, nranks = 1;
};

ncclResult_t bootstrap_get_unique_id(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  memset(id, 0, sizeof(*id));
  IdLayout L{};
  L.magic = kIdMagic;
  std::random_device rd;
  L.nonce = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)getpid();
  L.addr.sin_family = AF_INET;
  L.addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  L.addr.sin_port = 0;
  // NCCL_COMM_ID=<ip>:<port> (reference init.cc:93-106) pins the root address.
  const char* env = getenv("VCCL_COMM_ID");
  if (!env) env = getenv("NCCL_COMM_ID");
  if (env) {
    std::string s(env);
    auto c = s.rfind(':');
    if (c != std::string::npos) {
      inet_pton(AF_INET, s.substr(0, c).c_str(), &L.addr.sin_addr);
      L.addr.sin_port = htons((uint16_t)atoi(s.c_str() + c + 1));
    }
  }
  int lfd = socket(AF_INET, SOCK_STREAM, 0);
  if (lfd < 0) return ncclSystemError;
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (bind(lfd, (sockaddr*)&L.addr, sizeof(L.addr)) != 0 || listen(lfd, 128) != 0) {
    VWARN("bootstrap: bind/listen failed: %s", strerror(errno));
    close(lfd);
    return ncclSystemError;
  }
  socklen_t sl = sizeof(L.addr);
  getsockname(lfd, (sockaddr*)&L.addr, &sl);
  std::thread(root_main, lfd, L.nonce).detach();
  memcpy(id->internal, &L, sizeof(L));
  return ncclSuccess;
}

ncclResult_t bootstrap_init(const ncclUniqueId* id, int rank, int nranks, Bootstrap** out,
                            const std::atomic<bool>* abortReq) {
  IdLayout L;
  memcpy(&L, id->internal, sizeof(L));
  if (L.magic != kIdMagic) {
    VWARN("bootstrap: invalid unique id");
    return ncclInvalidArgument;
  }
  int fd = -1;
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::seconds(param_int("BOOTSTRAP_TIMEOUT", 600));
  for (;;) {
    fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return ncclSystemError;
    if (connect(fd, (sockaddr*)&L.addr, sizeof(L.addr)) == 0) break;
    close(fd);
    fd = -1;
    if (std::chrono::steady_clock::now() > deadline) {
      VWARN("bootstrap: cannot reach root");
      return ncclSystemError;
    }
    if (abortReq && abortReq->load()) {
      VWARN("bootstrap: aborted before the root was reached");
      return ncclRemoteError;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  set_nodelay(fd);
  Hello h{kHelloMagic, L.nonce, rank, nranks};
  if (!send_all(fd, &h, sizeof(h))) {
    close(fd);
    return ncclSystemError;
  }
  auto* b = new Bootstrap;
  b->fd = fd;
  b->rank = rank;
  b->nranks = nranks;
  *out = b;
  return ncclSuccess;
}

ncclResult_t bootstrap_allgather(Bootstrap* b, void* buf, size_t bytes) {
  uint64_t len = bytes;
  char* mine = (char*)buf + (size_t)b->rank * bytes;
  if (!send_all(b->fd, &len, sizeof(len)) || !send_all(b->fd, mine, bytes)) return ncclSystemError;
  if (!recv_all(b->fd, buf, bytes * (size_t)b->nranks)) return ncclSystemError;
  return ncclSuccess;
}

int bootstrap_fd(const Bootstrap* b) { return b ? b->fd : -1; }

ncclResult_t bootstrap_barrier(Bootstrap* b) {
  std::vector<char> tmp((size_t)b->nranks);
  return bootstrap_allgather(b, tmp.data(), 1);
}

// IPv4 address (network order) of the interface this rank reaches the root
// through: the address peers on other nodes can reach this rank at.
uint32_t bootstrap_local_ip(Bootstrap* b) {
  sockaddr_in a{};
  socklen_t sl = sizeof(a);
  if (!b || getsockname(b->fd, (sockaddr*)&a, &sl) != 0) return htonl(INADDR_LOOPBACK);
  return a.sin_addr.s_addr;
}

void bootstrap_close(Bootstrap* b) {
  if (!b) return;
  if (b->fd >= 0) close(b->fd);
  delete b;
}

}  // namespace vccl

extern "C" __attribute__((visibility("default"))) ncclResult_t vcclBootstrapAllGather(
    const ncclUniqueId* id, int rank, int nranks, void* buf, size_t bytesPerRank) {
  if (!id || !buf || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  vccl::Bootstrap* b = nullptr;
  ncclResult_t r = vccl::bootstrap_init(id, rank, nranks, &b);
  if (r != ncclSuccess) return r;
  r = vccl::bootstrap_allgather(b, buf, bytesPerRank);
  vccl::bootstrap_close(b);
  return r;
}
