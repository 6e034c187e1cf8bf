// Net transport: ring connections between nodes, staged through host-pinned
// buffers by a proxy thread pair over TCP.
//
// Reference role: the proxy thread and the socket / IB net transports
// (src/proxy.cc:914-971 progress loop, src/transport/net.cc:1293-1482
// sendProxyProgress / recvProxyProgress) without GPUDirect RDMA: the GPU
// writes a slot into host memory, the sender's proxy ships it, the receiver's
// proxy lands it in host memory the receiving GPU reads, credits flow back.
//
// MI355X design: the kernel does not know a connection is remote.  A net
// channel end is the same DevChannel the xGMI ring uses, with its pointers
// aimed at host-pinned (fine-grained, device-mapped) memory instead of the
// peer's HBM:
//   send end  sendFifo     -> staging slots here   (GPU writes, proxy sends)
//             nextRecvTail -> sendTail flag here   (GPU posts step s+1)
//             sendSizes    -> bytes of each slot   (GPU, before the tail)
//             sendHead     -> credit flag here     (proxy, from the peer)
//   recv end  recvFifo     -> landing slots here   (proxy recv()s, GPU reads)
//             recvTail     -> arrival flag here    (proxy, after a whole slot)
//             prevSendHead -> consumed flag here   (GPU, proxy forwards it)
// Counters are the ring's persistent step counters, so the proxy simply
// mirrors them across calls.  Wire format per connection (one TCP stream per
// channel and direction): data {uint64 bytes, bytes of slot payload} in step
// order one way, credits {uint64 head} the other way.
//
// Threads: one per connection end.  A send end ships posted slots (blocking
// sends) and applies credits read without blocking; a receive end lands
// slots and forwards the GPU's consumed counts as 8-byte credits.  A blocked
// data send never stops a receive end, and credits are tiny (a 4 MiB socket
// buffer holds half a million), so the ring of proxies cannot deadlock.  Socket
// failures raise the comm's error flag: the GPU's bounded spins end and
// ncclCommGetAsyncError reports ncclRemoteError.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <thread>

#include "core.h"

namespace vccl {

namespace {
constexpr uint64_t kNetHello = 0x5643434c4e455431ull;  // "VCCLNET1"

struct NetHello {
  uint64_t magic;
  int32_t rank, channel;
};

// Host flag block of one channel: each flag on its own 128-byte line.
struct alignas(128) Line {
  uint64_t v;
  char pad[120];
};
struct ChanFlags {
  Line sendTail;      // GPU: slots posted into the staging buffer
  Line sendHead;      // proxy: slots the remote receiver consumed
  Line recvTail;      // proxy: slots landed
  Line recvHead;      // GPU: slots consumed
  uint32_t sendSizes[kSteps];  // GPU: bytes posted per slot; kNetSizeUnset once shipped
  uint32_t recvSizes[kSteps];  // proxy: bytes landed per slot (the GPU checks them)
  char pad[128 - 2 * sizeof(uint32_t) * kSteps];
};

struct Conn {
  int ch = -1;
  int fd = -1;
  // VCCL_DEBUG_NET_SHORT_SLOT=b (test hook): ship the connection's first slot
  // of at least b bytes 16 bytes short, as a stale size would
  int64_t shortSlot = 0;
  char* buf = nullptr;       // kSteps slots, host pointer
  ChanFlags* flags = nullptr;
  uint64_t done = 0;         // send: slots shipped; recv: slots landed
  uint64_t credited = 0;     // recv: consumed count forwarded to the sender
};

uint64_t ld_acq(const uint64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
void st_rel(uint64_t* p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

}  // namespace

struct NetProxy {
  std::vector<Conn> send, recv;
  int64_t stride = 0;        // slot stride in bytes
  char* host = nullptr;      // one hipHostMalloc block: flags, then slots
  std::atomic<bool> stop{false};
  std::vector<std::thread> threads;  // one per connection end
  volatile int* errorFlag = nullptr;  // the comm's host-mapped error word
  std::atomic<uint64_t> bytesSent{0}, bytesRecv{0};
  int64_t sizeWaitS = 60;    // bound on a posted slot's size staying unset
};

namespace {

// Socket failures read as a lost peer (kErrSpinTimeout: ncclRemoteError); a
// slot size that is not valid, as kErrSlotSize (ncclInternalError).
void fail(NetProxy* P, const char* what, int ch, int word = kErrSpinTimeout) {
  if (!P->stop.load()) {
    if (word == kErrSpinTimeout) VWARN("net proxy: %s on channel %d: %s", what, ch, strerror(errno));
    else VWARN("net proxy: %s on channel %d", what, ch);
    *P->errorFlag = word;
  }
}

// Blocking I/O that gives up when the proxy is stopping.
bool io_all(NetProxy* P, int fd, void* p, size_t n, bool out) {
  char* c = (char*)p;
  while (n) {
    ssize_t k = out ? ::send(fd, c, n, MSG_NOSIGNAL) : ::recv(fd, c, n, 0);
    if (k > 0) {
      c += k;
      n -= (size_t)k;
      continue;
    }
    if (k < 0 && (errno == EINTR || errno == EAGAIN)) continue;
    return false;
  }
  (void)P;
  return true;
}

// One thread per connection end, so the staged rate scales with channels
// (one sending thread's socket copy tops out near 10 GB/s).
void idle_wait(bool busy, int* idle) {
  if (busy) *idle = 0;
  else if (++*idle > 256) std::this_thread::sleep_for(std::chrono::microseconds(20));
}

// Send end: ship every posted slot {bytes, payload} in step order; apply the
// receiver's credits (8-byte head values, read without blocking).
//
// Slot sizes carry the reference's sentinel (src/transport/net.cc:1250-1255,
// 1365-1367: a consumed slot's size is reset to -1 and the proxy sends only
// once it is valid): a shipped slot's size word goes back to kNetSizeUnset,
// so a size the GPU has not (yet) published is never shipped as a stale
// one.  The GPU releases the size before the tail (ring.hpp), so a valid
// size normally shows at once; one still unset after VCCL_SPIN_TIMEOUT_S, or
// a size past the slot stride, is an error (the comm's error word), never a
// clamped or short slot.  The credit that lets the GPU reuse the slot is
// applied by this same thread after the reset, so the reset cannot land on
// the next use of the slot.
void send_loop(NetProxy* P, Conn* c) {
  int idle = 0;
  uint64_t credit = 0;
  size_t have = 0;  // bytes of `credit` received so far
  while (!P->stop.load(std::memory_order_relaxed)) {
    bool busy = false;
    const uint64_t posted = ld_acq(&c->flags->sendTail.v);
    while (c->done < posted && !P->stop.load(std::memory_order_relaxed)) {
      const int slot = (int)(c->done % kSteps);
      uint32_t sz = __atomic_load_n(&c->flags->sendSizes[slot], __ATOMIC_ACQUIRE);
      if (sz == kNetSizeUnset) {
        const auto t0 = std::chrono::steady_clock::now();
        while ((sz = __atomic_load_n(&c->flags->sendSizes[slot], __ATOMIC_ACQUIRE)) == kNetSizeUnset &&
               !P->stop.load(std::memory_order_relaxed)) {
          if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(P->sizeWaitS)) {
            fail(P, "a posted slot's size never became valid", c->ch, kErrSlotSize);
            return;
          }
          std::this_thread::yield();
        }
        if (sz == kNetSizeUnset) return;  // stopping
      }
      if (sz > (uint64_t)P->stride) {
        fail(P, "a posted slot's size is past the slot stride", c->ch, kErrSlotSize);
        return;
      }
      uint64_t bytes = sz;
      if (c->shortSlot && (int64_t)bytes >= std::max<int64_t>(c->shortSlot, 32)) {
        bytes -= 16;  // test hook: a stale / short size, which the receiving kernel must refuse
        c->shortSlot = 0;
      }
      __atomic_store_n(&c->flags->sendSizes[slot], kNetSizeUnset, __ATOMIC_RELAXED);
      if (!io_all(P, c->fd, &bytes, sizeof(bytes), true) ||
          (bytes && !io_all(P, c->fd, c->buf + slot * P->stride, bytes, true))) {
        fail(P, "send", c->ch);
        return;
      }
      P->bytesSent += bytes;
      c->done++;
      busy = true;
    }
    for (;;) {
      const ssize_t k = ::recv(c->fd, (char*)&credit + have, sizeof(credit) - have, MSG_DONTWAIT);
      if (k > 0) {
        have += (size_t)k;
        if (have == sizeof(credit)) {
          st_rel(&c->flags->sendHead.v, credit);
          have = 0;
        }
        busy = true;
        continue;
      }
      if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) break;
      fail(P, "credit recv", c->ch);
      return;
    }
    idle_wait(busy, &idle);
  }
}

// Receive end: forward the GPU's consumed count as a credit; land each
// arriving slot whole, then raise the tail the GPU waits on.
void recv_loop(NetProxy* P, Conn* c) {
  int idle = 0;
  while (!P->stop.load(std::memory_order_relaxed)) {
    bool busy = false;
    const uint64_t head = ld_acq(&c->flags->recvHead.v);
    if (head > c->credited) {
      if (!io_all(P, c->fd, (void*)&head, sizeof(head), true)) {
        fail(P, "credit send", c->ch);
        return;
      }
      c->credited = head;
      busy = true;
    }
    pollfd pf{c->fd, POLLIN, 0};
    const int ready = poll(&pf, 1, 0);
    if (ready < 0 && errno != EINTR) {
      fail(P, "poll", c->ch);
      return;
    }
    if (ready > 0 && (pf.revents & (POLLIN | POLLHUP | POLLERR))) {
      uint64_t bytes = 0;
      if (!io_all(P, c->fd, &bytes, sizeof(bytes), false) || bytes > (uint64_t)P->stride ||
          (bytes && !io_all(P, c->fd, c->buf + (c->done % kSteps) * P->stride, bytes, false))) {
        fail(P, "recv", c->ch);
        return;
      }
      P->bytesRecv += bytes;
      // the landed byte count, before the tail (the kernel compares it with
      // the step's slice length, ring.hpp recv_size_ok)
      __atomic_store_n(&c->flags->recvSizes[c->done % kSteps], (uint32_t)bytes, __ATOMIC_RELAXED);
      c->done++;
      st_rel(&c->flags->recvTail.v, c->done);
      busy = true;
    }
    idle_wait(busy, &idle);
  }
}

int tcp_socket() {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd >= 0) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int sz = 4 << 20;
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
  }
  return fd;
}

}  // namespace

ncclResult_t net_listen(ncclComm* c, PeerMap* me) {
  int fd = tcp_socket();
  if (fd < 0) return ncclSystemError;
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = bootstrap_local_ip(c->bootstrap);
  a.sin_port = 0;
  socklen_t sl = sizeof(a);
  if (bind(fd, (sockaddr*)&a, sizeof(a)) != 0 || listen(fd, 2 * kMaxChannels) != 0 ||
      getsockname(fd, (sockaddr*)&a, &sl) != 0) {
    VWARN("net proxy: bind/listen failed: %s", strerror(errno));
    close(fd);
    return ncclSystemError;
  }
  c->netListenFd = fd;
  me->netIp = a.sin_addr.s_addr;
  me->netPort = a.sin_port;
  return ncclSuccess;
}

ncclResult_t net_connect(ncclComm* c, const std::vector<std::vector<int>>& rings,
                         std::vector<DevChannel>& chans, const std::vector<char>& netPeer) {
  const int n = c->nRanks, nch = c->nChannels, nRings = (int)rings.size();
  auto* P = new NetProxy;
  c->net = P;
  P->errorFlag = c->errorFlag;
  P->stride = slot_stride(c->slotBytes);
  std::vector<int> sendCh, recvCh;  // channels with a net send / recv end
  std::vector<int> nextOf(nch), prevOf(nch);
  for (int ch = 0; ch < nch; ch++) {
    const auto& ring = rings[ch % nRings];
    const int pos = (int)(std::find(ring.begin(), ring.end(), c->rank) - ring.begin());
    nextOf[ch] = ring[(pos + 1) % n];
    prevOf[ch] = ring[(pos + n - 1) % n];
    if (netPeer[nextOf[ch]]) sendCh.push_back(ch);
    if (netPeer[prevOf[ch]]) recvCh.push_back(ch);
  }
  const size_t nConn = sendCh.size() + recvCh.size();
  const size_t flagBytes = (size_t)nch * sizeof(ChanFlags);
  const size_t bytes = flagBytes + nConn * kSteps * (size_t)P->stride;
  HIPCHECK(hipHostMalloc((void**)&P->host, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  memset(P->host, 0, flagBytes);
  for (int ch = 0; ch < nch; ch++)
    for (int k = 0; k < kSteps; k++) ((ChanFlags*)P->host)[ch].sendSizes[k] = kNetSizeUnset;
  P->sizeWaitS = std::max<int64_t>(1, param_int("SPIN_TIMEOUT_S", 60));
  const int64_t shortSlot = param_int("DEBUG_NET_SHORT_SLOT", 0);
  char* dev = nullptr;
  HIPCHECK(hipHostGetDevicePointer((void**)&dev, P->host, 0));
  auto devp = [&](void* h) { return dev + ((char*)h - P->host); };
  ChanFlags* flags = (ChanFlags*)P->host;
  char* slots = P->host + flagBytes;

  // Connect my send ends (the peer's backlog completes them before it
  // accepts), then accept my receive ends and match them by their hello.
  for (int ch : sendCh) {
    const PeerMap& p = c->peers[nextOf[ch]];
    Conn k;
    k.ch = ch;
    k.fd = tcp_socket();
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = p.netIp;
    a.sin_port = p.netPort;
    NetHello h{kNetHello, c->rank, ch};
    if (k.fd < 0 || connect(k.fd, (sockaddr*)&a, sizeof(a)) != 0 ||
        !io_all(P, k.fd, &h, sizeof(h), true)) {
      VWARN("net proxy: connect to rank %d (channel %d) failed: %s", nextOf[ch], ch, strerror(errno));
      if (k.fd >= 0) close(k.fd);
      return ncclSystemError;
    }
    k.buf = slots;
    slots += kSteps * P->stride;
    k.flags = &flags[ch];
    k.shortSlot = shortSlot;
    P->send.push_back(k);
  }
  for (size_t i = 0; i < recvCh.size(); i++) {
    pollfd pf{c->netListenFd, POLLIN, 0};
    const int timeoutMs = (int)param_int("NET_CONNECT_TIMEOUT_S", 300) * 1000;
    if (poll(&pf, 1, timeoutMs) != 1) {
      VWARN("net proxy: rank %d timed out accepting connections", c->rank);
      return ncclSystemError;
    }
    int fd = accept(c->netListenFd, nullptr, nullptr);
    NetHello h{};
    if (fd < 0 || !io_all(P, fd, &h, sizeof(h), false) || h.magic != kNetHello ||
        std::find(recvCh.begin(), recvCh.end(), h.channel) == recvCh.end() ||
        h.rank != prevOf[h.channel]) {
      VWARN("net proxy: bad connection on rank %d", c->rank);
      if (fd >= 0) close(fd);
      return ncclSystemError;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    Conn k;
    k.ch = h.channel;
    k.fd = fd;
    k.buf = slots;
    slots += kSteps * P->stride;
    k.flags = &flags[h.channel];
    P->recv.push_back(k);
  }
  close(c->netListenFd);
  c->netListenFd = -1;

  // Aim the channel ends at the staging memory.
  for (const Conn& k : P->send) {
    DevChannel& d = chans[k.ch];
    d.sendFifo = devp(k.buf);
    d.nextRecvTail = (uint64_t*)devp(&k.flags->sendTail.v);
    d.sendHead = (uint64_t*)devp(&k.flags->sendHead.v);
    d.sendSizes = (uint32_t*)devp(k.flags->sendSizes);
  }
  for (const Conn& k : P->recv) {
    DevChannel& d = chans[k.ch];
    d.recvFifo = devp(k.buf);
    d.recvTail = (uint64_t*)devp(&k.flags->recvTail.v);
    d.prevSendHead = (uint64_t*)devp(&k.flags->recvHead.v);
    d.recvSizes = (const uint32_t*)devp(k.flags->recvSizes);
  }
  for (Conn& k : P->send) P->threads.emplace_back(send_loop, P, &k);
  for (Conn& k : P->recv) P->threads.emplace_back(recv_loop, P, &k);
  VINFO("rank %d: net proxy up, %zu send / %zu recv connections", c->rank, P->send.size(),
        P->recv.size());
  return ncclSuccess;
}

void net_stop(ncclComm* c) {
  if (c->netListenFd >= 0) close(c->netListenFd);
  c->netListenFd = -1;
  NetProxy* P = c->net;
  if (!P) return;
  P->stop.store(true);
  for (Conn& k : P->send) shutdown(k.fd, SHUT_RDWR);
  for (Conn& k : P->recv) shutdown(k.fd, SHUT_RDWR);
  for (std::thread& t : P->threads) t.join();
  for (Conn& k : P->send) close(k.fd);
  for (Conn& k : P->recv) close(k.fd);
  if (P->host) (void)hipHostFree(P->host);
  delete P;
  c->net = nullptr;
}

}  // namespace vccl

// Bytes moved by this comm's net proxy so far (diagnostics / tests).
extern "C" __attribute__((visibility("default"))) ncclResult_t vcclCommNetStats(
    ncclComm_t comm, uint64_t* sent, uint64_t* received, int* connections) {
  if (vccl::comm_check(comm, "vcclCommNetStats") != ncclSuccess) return ncclInvalidArgument;
  const vccl::NetProxy* P = comm->net;
  if (sent) *sent = P ? P->bytesSent.load() : 0;
  if (received) *received = P ? P->bytesRecv.load() : 0;
  if (connections) *connections = P ? (int)(P->send.size() + P->recv.size()) : 0;
  return ncclSuccess;
}
