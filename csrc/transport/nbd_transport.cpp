// nbd_transport.cpp — ZMTP/3.1 DEALER/ROUTER transport with an epoll I/O thread.
// See nbd_transport.h for the design summary.
#include "nbd_transport.h"

#include <arpa/inet.h>
#include <endian.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;
thread_local std::string g_err;

int fail(const std::string& m) {
  g_err = m;
  return -1;
}
std::string errstr(const char* what) { return std::string(what) + ": " + std::strerror(errno); }

constexpr uint64_t TOK_WAKE = 1;
constexpr uint64_t TOK_CAP0 = 2;  // + stream index (0 = stdout, 1 = stderr)
constexpr uint64_t TOK_FIRST = 16;
constexpr size_t kMaxFrame = (size_t)1 << 36;  // 64 GiB sanity bound
constexpr int kHandshakeTimeoutMs = 10000;

struct Msg {
  int kind = NBD_KIND_MSG;
  int event = 0;
  std::vector<std::string> frames;
};

// Growable read buffer: [pos, len) holds unparsed bytes.
struct RBuf {
  std::unique_ptr<char[]> d;
  size_t cap = 0, len = 0, pos = 0;
  void reserve_tail(size_t n) {  // ensure n writable bytes after len
    if (len + n <= cap) return;
    if (pos > 0) {  // compact first
      std::memmove(d.get(), d.get() + pos, len - pos);
      len -= pos;
      pos = 0;
      if (len + n <= cap) return;
    }
    size_t nc = std::max<size_t>(cap ? cap * 2 : 65536, len + n);
    std::unique_ptr<char[]> nd(new char[nc]);
    if (len) std::memcpy(nd.get(), d.get(), len);
    d.swap(nd);
    cap = nc;
  }
  void consumed() {
    if (pos == len) pos = len = 0;
  }
};

enum class PState { Connecting, Greeting, Handshake, Active, Closed };

struct Peer {
  uint64_t tok = 0;
  int fd = -1;
  std::atomic<PState> st{PState::Greeting};
  int connect_idx = -1;  // DEALER: index of the ConnectRec that owns this peer
  RBuf rb;
  size_t want = 0;  // bytes needed to complete the frame being parsed (reservation hint)
  std::vector<std::string> cur;
  std::mutex omu;
  std::condition_variable ocv;
  std::deque<std::string> outq;
  size_t ooff = 0, oqbytes = 0;
  bool epollout = false;
  bool closed = false;  // guarded by omu
  std::string identity, peer_type;
  int minor = 0;
  Clock::time_point created, last_rx, last_ping;
};
using PeerP = std::shared_ptr<Peer>;

struct ConnectRec {
  std::string ep;
  uint64_t peer_tok = 0;
  Clock::time_point next_try;
};
struct Listener {
  int fd = -1;
  std::string ipc_path;
};
struct Capture {
  int rfd = -1, saved = -1, target = -1;
  std::string buf;
  Clock::time_point first;
};

struct Addr {
  bool ipc = false;
  std::string path, host, port;
};

bool parse_ep(const std::string& ep, Addr& a) {
  if (ep.rfind("tcp://", 0) == 0) {
    std::string rest = ep.substr(6);
    size_t c = rest.rfind(':');
    if (c == std::string::npos) return false;
    a.host = rest.substr(0, c);
    a.port = rest.substr(c + 1);
    if (a.host.size() >= 2 && a.host.front() == '[' && a.host.back() == ']')
      a.host = a.host.substr(1, a.host.size() - 2);
    if (a.port == "*") a.port = "0";
    return !a.port.empty();
  }
  if (ep.rfind("ipc://", 0) == 0) {
    a.ipc = true;
    a.path = ep.substr(6);
    return !a.path.empty() && a.path.size() < sizeof(sockaddr_un::sun_path);
  }
  return false;
}

std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

void put_frame(std::string& out, const void* p, size_t n, bool more, bool cmd) {
  uint8_t flags = (uint8_t)((more ? 1 : 0) | (cmd ? 4 : 0));
  if (n > 255) {
    flags |= 2;
    out.push_back((char)flags);
    uint64_t be = htobe64((uint64_t)n);
    out.append(reinterpret_cast<const char*>(&be), 8);
  } else {
    out.push_back((char)flags);
    out.push_back((char)(uint8_t)n);
  }
  if (n) out.append(static_cast<const char*>(p), n);
}

void put_prop(std::string& body, const std::string& name, const std::string& value) {
  body.push_back((char)(uint8_t)name.size());
  body += name;
  uint32_t be = htobe32((uint32_t)value.size());
  body.append(reinterpret_cast<const char*>(&be), 4);
  body += value;
}

std::string command(const std::string& name, const std::string& data) {
  std::string body;
  body.push_back((char)(uint8_t)name.size());
  body += name;
  body += data;
  std::string out;
  put_frame(out, body.data(), body.size(), false, true);
  return out;
}

std::string greeting() {
  std::string g(64, '\0');
  g[0] = (char)0xFF;
  g[8] = 0x01;
  g[9] = 0x7F;
  g[10] = 3;  // major
  g[11] = 1;  // minor: ZMTP/3.1 (PING/PONG)
  std::memcpy(&g[12], "NULL", 4);
  g[32] = 0;  // as-server (unused by NULL)
  return g;
}

bool compatible(int mytype, const std::string& peer) {
  if (mytype == NBD_ROUTER) return peer == "DEALER" || peer == "REQ" || peer == "ROUTER";
  return peer == "ROUTER" || peer == "REP" || peer == "DEALER";
}

}  // namespace

struct nbd_msg {
  Msg m;
};

struct nbd_socket {
  int type;
  // options: numeric ones are atomics (set from API threads, read by the I/O thread);
  // string ones are guarded by optmu and copied out under it.
  std::mutex optmu;
  std::string identity, token, sig_prefix;
  std::atomic<int> hb_ivl_ms{0}, hb_timeout_ms{0}, reconnect_ivl_ms{100};
  std::atomic<bool> mandatory{false};
  std::atomic<int64_t> flush_us{2000};
  std::atomic<size_t> stream_max{1 << 16};
  std::atomic<size_t> hwm{0};
  // latency options: a receiver that expects a reply within tens of microseconds polls instead
  // of sleeping on a futex / in epoll_wait (each sleep -> wake hop costs 5-30 us on an idle core)
  std::atomic<int64_t> recv_spin_us{0}, io_spin_us{0};

  int ep = -1, evfd = -1;
  std::thread io;
  std::atomic<bool> stop{false};
  std::atomic<bool> closing{false};
  std::atomic<int> users{0};

  std::mutex mu;  // peers / routing / listeners / connects / pending
  std::map<uint64_t, PeerP> peers;
  std::map<std::string, PeerP> by_id;  // active peers by identity
  std::vector<PeerP> active;           // active peers (DEALER round-robin)
  std::map<uint64_t, Listener> listeners;
  std::vector<ConnectRec> connects;
  std::deque<std::string> pending;  // DEALER: queued while no peer is active
  size_t rr = 0;
  uint64_t next_tok = TOK_FIRST;
  uint32_t next_anon = 1;

  std::mutex imu;
  std::condition_variable icv;
  std::deque<Msg*> inbox;
  bool inbox_closed = false;
  std::atomic<size_t> inbox_n{0};     // inbox.size(), readable without imu (receiver spin)
  std::atomic<bool> wake_pending{false};  // set by nbd_wake_recv, consumed by one receive call

  std::mutex cmu;  // capture state; lock order: cmu -> mu -> Peer::omu
  Capture cap[2];
  std::string stream_hdr[2];

  explicit nbd_socket(int t) : type(t) {}

  // ---------------------------------------------------------------- plumbing
  void wake() {
    uint64_t one = 1;
    ssize_t r = ::write(evfd, &one, 8);
    (void)r;
  }

  // Receiver-side poll (NBD_OPT_RECV_SPIN_US): up to recv_spin_us (bounded by the call's
  // timeout) watching inbox_n / wake_pending, so a reply that lands within the window is taken
  // without a futex sleep.
  void spin_for_inbox(int timeout_ms) {
    int64_t us = recv_spin_us.load(std::memory_order_relaxed);
    if (timeout_ms >= 0) us = std::min<int64_t>(us, (int64_t)timeout_ms * 1000);
    if (us <= 0) return;
    const auto end = Clock::now() + std::chrono::microseconds(us);
    for (int i = 0;; ++i) {
      if (inbox_n.load(std::memory_order_acquire) > 0 || closing.load() || wake_pending.load()) break;
      __builtin_ia32_pause();
      if ((i & 63) == 63 && Clock::now() >= end) break;
    }
  }

  void push_inbox(Msg* m) {
    {
      std::lock_guard<std::mutex> lk(imu);
      if (inbox_closed) {
        delete m;
        return;
      }
      inbox.push_back(m);
      inbox_n.store(inbox.size(), std::memory_order_release);
    }
    icv.notify_one();
  }

  void push_event(int code, const std::string& ident) {
    Msg* m = new Msg;
    m->kind = NBD_KIND_EVENT;
    m->event = code;
    m->frames.push_back(ident);
    push_inbox(m);
  }

  void epoll_mod(Peer& p) {  // requires p.omu
    epoll_event ev{};
    ev.events = EPOLLIN | (p.epollout ? (uint32_t)EPOLLOUT : 0u);
    ev.data.u64 = p.tok;
    epoll_ctl(ep, EPOLL_CTL_MOD, p.fd, &ev);
  }

  // Write as much of the queue as the kernel takes.  Requires p.omu.  false = fatal error.
  bool flush_locked(Peer& p) {
    while (!p.outq.empty()) {
      iovec iov[64];
      int n = 0;
      size_t off = p.ooff;
      for (auto it = p.outq.begin(); it != p.outq.end() && n < 64; ++it, ++n) {
        iov[n].iov_base = const_cast<char*>(it->data()) + off;
        iov[n].iov_len = it->size() - off;
        off = 0;
      }
      msghdr mh{};
      mh.msg_iov = iov;
      mh.msg_iovlen = (size_t)n;
      ssize_t w = ::sendmsg(p.fd, &mh, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        return false;
      }
      size_t left = (size_t)w;
      p.oqbytes -= left;
      while (left > 0) {
        size_t rem = p.outq.front().size() - p.ooff;
        if (left >= rem) {
          left -= rem;
          p.outq.pop_front();
          p.ooff = 0;
        } else {
          p.ooff += left;
          left = 0;
        }
      }
    }
    bool need = !p.outq.empty();
    if (need != p.epollout) {
      p.epollout = need;
      epoll_mod(p);
    }
    p.ocv.notify_all();
    return true;
  }

  // Queue bytes for a peer and try to write them right away from the calling thread.
  int enqueue(const PeerP& p, std::string&& data, bool may_block) {
    std::unique_lock<std::mutex> lk(p->omu);
    const size_t lim = hwm.load();
    if (may_block && lim > 0) {
      while (!p->closed && !closing.load() && p->oqbytes > lim) p->ocv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(50));
    }
    if (p->closed) return fail("EPIPE: peer connection closed");
    p->oqbytes += data.size();
    p->outq.push_back(std::move(data));
    if (!p->epollout && p->fd >= 0 && p->st != PState::Connecting) {
      if (!flush_locked(*p)) {
        // The I/O thread sees the error (EPOLLERR/HUP) and closes the peer.
        p->epollout = true;
        epoll_mod(*p);
      }
    }
    return 0;
  }

  // Route an encoded message.  frames_for_router: identity is separate.
  int route(const std::string* ident, std::string&& data, bool may_block) {
    PeerP p;
    {
      std::lock_guard<std::mutex> lk(mu);
      if (type == NBD_ROUTER) {
        auto it = by_id.find(*ident);
        if (it == by_id.end()) {
          if (mandatory) return fail("EHOSTUNREACH: no peer with this identity");
          return 0;  // silently dropped, like libzmq's ROUTER
        }
        p = it->second;
      } else {
        if (active.empty()) {
          pending.push_back(std::move(data));
          return 0;
        }
        p = active[rr++ % active.size()];
      }
    }
    return enqueue(p, std::move(data), may_block);
  }

  static std::string encode(int nframes, const void* const* ptrs, const size_t* lens, int first) {
    size_t total = 0;
    for (int i = first; i < nframes; ++i) total += lens[i] + 9;
    std::string out;
    out.reserve(total);
    for (int i = first; i < nframes; ++i) put_frame(out, ptrs[i], lens[i], i + 1 < nframes, false);
    return out;
  }

  // ---------------------------------------------------------------- peers
  PeerP add_peer(int fd, PState st, int connect_idx) {  // I/O thread
    auto p = std::make_shared<Peer>();
    p->fd = fd;
    p->st = st;
    p->connect_idx = connect_idx;
    p->created = p->last_rx = p->last_ping = Clock::now();
    {
      std::lock_guard<std::mutex> lk(mu);
      p->tok = next_tok++;
      peers[p->tok] = p;
      if (connect_idx >= 0) connects[(size_t)connect_idx].peer_tok = p->tok;
    }
    epoll_event ev{};
    ev.events = EPOLLIN | (st == PState::Connecting ? (uint32_t)EPOLLOUT : 0u);
    ev.data.u64 = p->tok;
    p->epollout = (st == PState::Connecting);
    epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
    if (st == PState::Greeting) enqueue(p, greeting(), false);
    return p;
  }

  void close_peer(const PeerP& p, int code) {  // I/O thread
    bool was_active;
    {
      std::lock_guard<std::mutex> lk(p->omu);
      if (p->closed) return;
      p->closed = true;
      epoll_ctl(ep, EPOLL_CTL_DEL, p->fd, nullptr);
      ::close(p->fd);
      p->fd = -1;
      p->ocv.notify_all();
    }
    was_active = (p->st == PState::Active);
    p->st = PState::Closed;
    {
      std::lock_guard<std::mutex> lk(mu);
      peers.erase(p->tok);
      auto it = by_id.find(p->identity);
      if (was_active && it != by_id.end() && it->second == p) by_id.erase(it);
      active.erase(std::remove(active.begin(), active.end(), p), active.end());
      if (p->connect_idx >= 0 && (size_t)p->connect_idx < connects.size()) {
        auto& rec = connects[(size_t)p->connect_idx];
        if (rec.peer_tok == p->tok) {
          rec.peer_tok = 0;
          rec.next_try = Clock::now() + std::chrono::milliseconds(reconnect_ivl_ms.load());
        }
      }
    }
    if (was_active)
      push_event(code ? code : NBD_EV_DISCONNECTED, p->identity);
    else if (code && code != NBD_EV_DISCONNECTED)
      push_event(code, p->identity);
  }

  void send_ready(const PeerP& p) {
    std::string props, id, tok;
    {
      std::lock_guard<std::mutex> lk(optmu);
      id = identity;
      tok = token;
    }
    put_prop(props, "Socket-Type", type == NBD_ROUTER ? "ROUTER" : "DEALER");
    put_prop(props, "Identity", id);
    if (!tok.empty()) put_prop(props, "X-Nbd-Token", tok);
    enqueue(p, command("READY", props), false);
  }

  // returns 0 ok, or an event code to close with
  int on_command(const PeerP& p, const char* d, size_t n) {
    if (n < 1) return NBD_EV_HANDSHAKE_FAILED;
    size_t nl = (uint8_t)d[0];
    if (1 + nl > n) return NBD_EV_HANDSHAKE_FAILED;
    std::string name(d + 1, nl);
    const char* data = d + 1 + nl;
    size_t dn = n - 1 - nl;
    if (name == "READY") {
      if (p->st != PState::Handshake) return NBD_EV_HANDSHAKE_FAILED;
      std::string ptype, pid, ptok;
      bool has_tok = false;
      size_t i = 0;
      while (i < dn) {
        size_t kl = (uint8_t)data[i++];
        if (i + kl + 4 > dn) return NBD_EV_HANDSHAKE_FAILED;
        std::string key = lower(std::string(data + i, kl));
        i += kl;
        uint32_t be;
        std::memcpy(&be, data + i, 4);
        i += 4;
        size_t vl = be32toh(be);
        if (i + vl > dn) return NBD_EV_HANDSHAKE_FAILED;
        std::string val(data + i, vl);
        i += vl;
        if (key == "socket-type") ptype = val;
        else if (key == "identity") pid = val;
        else if (key == "x-nbd-token") { ptok = val; has_tok = true; }
      }
      if (!compatible(type, ptype)) {
        enqueue(p, command("ERROR", std::string(1, (char)22) + "Incompatible socket"), false);
        return NBD_EV_HANDSHAKE_FAILED;
      }
      std::string mytok;
      {
        std::lock_guard<std::mutex> lk(optmu);
        mytok = token;
      }
      if (!mytok.empty() && (!has_tok || ptok != mytok)) {
        enqueue(p, command("ERROR", std::string(1, (char)13) + "Invalid token"), false);
        return NBD_EV_AUTH_FAILED;
      }
      p->peer_type = ptype;
      PeerP old;
      {
        std::lock_guard<std::mutex> lk(mu);
        if (pid.empty() || pid[0] == '\0') {
          uint32_t be = htobe32(next_anon++);
          pid = std::string(1, '\0') + std::string(reinterpret_cast<char*>(&be), 4);
        }
        p->identity = pid;
        p->st = PState::Active;
        if (type == NBD_ROUTER) {
          auto it = by_id.find(pid);
          if (it != by_id.end()) old = it->second;  // handover: newest connection wins
          by_id[pid] = p;
        }
        active.push_back(p);
        if (type == NBD_DEALER && !pending.empty()) {
          std::lock_guard<std::mutex> lk2(p->omu);
          for (auto& s : pending) {
            p->oqbytes += s.size();
            p->outq.push_back(std::move(s));
          }
          pending.clear();
          if (!p->epollout) flush_locked(*p);
        }
      }
      if (old) close_peer(old, NBD_EV_DISCONNECTED);
      push_event(NBD_EV_CONNECTED, pid);
      return 0;
    }
    if (name == "ERROR") return NBD_EV_HANDSHAKE_FAILED;
    if (name == "PING") {
      std::string ctx;
      if (dn > 2) ctx.assign(data + 2, std::min<size_t>(dn - 2, 16));
      enqueue(p, command("PONG", ctx), false);
      return 0;
    }
    return 0;  // PONG and unknown commands are ignored
  }

  void deliver(const PeerP& p) {
    Msg* m = new Msg;
    if (type == NBD_ROUTER) m->frames.push_back(p->identity);
    for (auto& f : p->cur) m->frames.push_back(std::move(f));
    p->cur.clear();
    std::string prefix;
    {
      std::lock_guard<std::mutex> lk(optmu);
      prefix = sig_prefix;
    }
    if (!prefix.empty()) {
      size_t k = (type == NBD_ROUTER) ? 1 : 0;
      if (m->frames.size() > k && m->frames[k].compare(0, prefix.size(), prefix) == 0) ::kill(::getpid(), SIGINT);
    }
    push_inbox(m);
  }

  // Parse everything buffered.  Returns 0 or an event code to close with.
  int parse(const PeerP& p) {
    RBuf& b = p->rb;
    for (;;) {
      size_t avail = b.len - b.pos;
      const uint8_t* s = reinterpret_cast<const uint8_t*>(b.d.get()) + b.pos;
      if (p->st == PState::Greeting) {
        if (avail >= 1 && s[0] != 0xFF) return NBD_EV_HANDSHAKE_FAILED;
        if (avail < 64) return 0;
        if (s[9] != 0x7F || s[10] < 3) return NBD_EV_HANDSHAKE_FAILED;
        p->minor = s[10] > 3 ? 1 : s[11];
        if (std::memcmp(s + 12, "NULL", 4) != 0 || s[16] != 0) return NBD_EV_HANDSHAKE_FAILED;
        b.pos += 64;
        p->st = PState::Handshake;
        send_ready(p);
        continue;
      }
      if (avail < 2) {
        p->want = 0;
        b.consumed();
        return 0;
      }
      uint8_t flags = s[0];
      if (flags & ~7u) return NBD_EV_HANDSHAKE_FAILED;
      size_t hdr, size;
      if (flags & 2) {
        if (avail < 9) return 0;
        uint64_t be;
        std::memcpy(&be, s + 1, 8);
        size = (size_t)be64toh(be);
        hdr = 9;
      } else {
        size = s[1];
        hdr = 2;
      }
      if (size > kMaxFrame) return NBD_EV_HANDSHAKE_FAILED;
      if (avail < hdr + size) {
        p->want = hdr + size - avail;
        return 0;
      }
      const char* body = reinterpret_cast<const char*>(s) + hdr;
      b.pos += hdr + size;
      if (flags & 4) {
        int rc = on_command(p, body, size);
        if (rc) return rc;
      } else {
        if (p->st != PState::Active) return NBD_EV_HANDSHAKE_FAILED;
        p->cur.emplace_back(body, size);
        if (!(flags & 1)) deliver(p);
      }
    }
  }

  void on_peer(uint64_t tok, uint32_t events) {
    PeerP p;
    {
      std::lock_guard<std::mutex> lk(mu);
      auto it = peers.find(tok);
      if (it == peers.end()) return;
      p = it->second;
    }
    if (p->st == PState::Connecting) {
      if (!(events & (EPOLLOUT | EPOLLERR | EPOLLHUP))) return;
      int err = 0;
      socklen_t el = sizeof(err);
      getsockopt(p->fd, SOL_SOCKET, SO_ERROR, &err, &el);
      if (err != 0) {
        close_peer(p, 0);
        return;
      }
      {
        std::lock_guard<std::mutex> lk(p->omu);
        p->st = PState::Greeting;
        p->epollout = false;
        epoll_mod(*p);
      }
      enqueue(p, greeting(), false);
      return;
    }
    if (events & EPOLLIN || events & (EPOLLERR | EPOLLHUP)) {
      for (;;) {
        size_t chunk = std::max<size_t>(65536, std::min<size_t>(p->want, (size_t)64 << 20));
        p->rb.reserve_tail(chunk);
        ssize_t r = ::recv(p->fd, p->rb.d.get() + p->rb.len, p->rb.cap - p->rb.len, 0);
        if (r > 0) {
          p->rb.len += (size_t)r;
          p->last_rx = Clock::now();
          int rc = parse(p);
          if (rc) {
            close_peer(p, rc);
            return;
          }
          continue;
        }
        if (r == 0) {
          close_peer(p, NBD_EV_DISCONNECTED);
          return;
        }
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        close_peer(p, NBD_EV_DISCONNECTED);
        return;
      }
    }
    if (events & EPOLLOUT) {
      std::lock_guard<std::mutex> lk(p->omu);
      if (!p->closed && !flush_locked(*p)) {
        // handled by the read side on the next EPOLLERR/HUP
      }
    }
  }

  void on_accept(uint64_t tok) {
    int lfd;
    bool ipc;
    {
      std::lock_guard<std::mutex> lk(mu);
      auto it = listeners.find(tok);
      if (it == listeners.end()) return;
      lfd = it->second.fd;
      ipc = !it->second.ipc_path.empty();
    }
    for (;;) {
      int fd = ::accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) {
        if (errno == EINTR) continue;
        return;
      }
      if (!ipc) {
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      }
      add_peer(fd, PState::Greeting, -1);
    }
  }

  void try_connect(size_t idx) {  // I/O thread
    Addr a;
    std::string epstr;
    {
      std::lock_guard<std::mutex> lk(mu);
      epstr = connects[idx].ep;
    }
    parse_ep(epstr, a);
    int fd = -1, rc = -1;
    if (a.ipc) {
      fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      sockaddr_un sa{};
      sa.sun_family = AF_UNIX;
      std::strncpy(sa.sun_path, a.path.c_str(), sizeof(sa.sun_path) - 1);
      rc = ::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa));
    } else {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_UNSPEC;
      hints.ai_socktype = SOCK_STREAM;
      if (getaddrinfo(a.host.c_str(), a.port.c_str(), &hints, &res) == 0 && res) {
        fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
        freeaddrinfo(res);
      }
    }
    if (fd >= 0 && (rc == 0 || errno == EINPROGRESS || errno == EAGAIN)) {
      // AF_UNIX reports EAGAIN when the backlog is full; treat like in-progress.
      if (rc == 0) add_peer(fd, PState::Greeting, (int)idx);
      else if (errno == EINPROGRESS) add_peer(fd, PState::Connecting, (int)idx);
      else {
        ::close(fd);
        std::lock_guard<std::mutex> lk(mu);
        connects[idx].next_try = Clock::now() + std::chrono::milliseconds(reconnect_ivl_ms.load());
      }
      return;
    }
    if (fd >= 0) ::close(fd);
    std::lock_guard<std::mutex> lk(mu);
    connects[idx].next_try = Clock::now() + std::chrono::milliseconds(reconnect_ivl_ms.load());
  }

  // ---------------------------------------------------------------- capture
  void emit_locked(int k) {  // requires cmu
    Capture& c = cap[k];
    if (c.buf.empty()) return;
    const std::string& h = stream_hdr[k];
    std::string out;
    out.reserve(h.size() + c.buf.size() + 20);
    put_frame(out, h.data(), h.size(), true, false);
    put_frame(out, c.buf.data(), c.buf.size(), false, false);
    c.buf.clear();
    route(nullptr, std::move(out), false);
  }

  void drain_locked(int k) {  // requires cmu
    Capture& c = cap[k];
    if (c.rfd < 0) return;
    char tmp[65536];
    for (;;) {
      ssize_t r = ::read(c.rfd, tmp, sizeof(tmp));
      if (r > 0) {
        if (c.buf.empty()) c.first = Clock::now();
        c.buf.append(tmp, (size_t)r);
        if (c.buf.size() >= stream_max) emit_locked(k);
        continue;
      }
      if (r < 0 && errno == EINTR) continue;
      break;
    }
  }

  // ---------------------------------------------------------------- I/O loop
  int next_timeout_ms() {
    int t = -1;
    auto now = Clock::now();
    {
      std::lock_guard<std::mutex> lk(mu);
      bool timers = false;
      for (auto& c : connects)
        if (c.peer_tok == 0) timers = true;
      for (auto& kv : peers)
        if (kv.second->st != PState::Active) timers = true;
      if (timers) t = 50;
      if ((hb_ivl_ms > 0 || hb_timeout_ms > 0) && !peers.empty()) {
        const int ivl = hb_ivl_ms.load(), tmo = hb_timeout_ms.load();
        int h = std::max(10, std::min(ivl > 0 ? ivl : 1000, tmo > 0 ? tmo : 1000) / 4);
        t = t < 0 ? h : std::min(t, h);
      }
    }
    {
      std::lock_guard<std::mutex> lk(cmu);
      for (auto& c : cap) {
        if (c.buf.empty()) continue;
        auto due = c.first + std::chrono::microseconds(flush_us.load());
        int ms = (int)std::chrono::duration_cast<std::chrono::milliseconds>(due - now).count();
        ms = std::max(ms, 0);
        if (due > now && ms == 0) ms = 1;
        t = t < 0 ? ms : std::min(t, ms);
      }
    }
    return t;
  }

  void timers() {
    auto now = Clock::now();
    // reconnects
    std::vector<size_t> todo;
    std::vector<PeerP> snapshot;
    {
      std::lock_guard<std::mutex> lk(mu);
      if (!stop)
        for (size_t i = 0; i < connects.size(); ++i)
          if (connects[i].peer_tok == 0 && now >= connects[i].next_try) todo.push_back(i);
      for (auto& kv : peers) snapshot.push_back(kv.second);
    }
    for (size_t i : todo) try_connect(i);
    for (auto& p : snapshot) {
      if (p->st != PState::Active) {
        auto age = std::chrono::duration_cast<std::chrono::milliseconds>(now - p->created).count();
        if (p->st != PState::Closed && age > kHandshakeTimeoutMs) close_peer(p, NBD_EV_HANDSHAKE_FAILED);
        continue;
      }
      if (hb_timeout_ms > 0 &&
          std::chrono::duration_cast<std::chrono::milliseconds>(now - p->last_rx).count() > hb_timeout_ms) {
        close_peer(p, NBD_EV_HEARTBEAT_TIMEOUT);
        continue;
      }
      if (hb_ivl_ms > 0 && p->minor >= 1 &&
          std::chrono::duration_cast<std::chrono::milliseconds>(now - p->last_ping).count() >= hb_ivl_ms) {
        p->last_ping = now;
        uint16_t ttl = htobe16((uint16_t)std::min(65535, hb_timeout_ms.load() / 100));
        enqueue(p, command("PING", std::string(reinterpret_cast<char*>(&ttl), 2)), false);
      }
    }
    {
      std::lock_guard<std::mutex> lk(cmu);
      for (int k = 0; k < 2; ++k) {
        Capture& c = cap[k];
        if (!c.buf.empty() && now - c.first >= std::chrono::microseconds(flush_us.load())) emit_locked(k);
      }
    }
  }

  void loop() {
    sigset_t all;
    sigfillset(&all);
    pthread_sigmask(SIG_BLOCK, &all, nullptr);  // signals belong to the application threads
    epoll_event evs[64];
    auto active_until = Clock::now(), last_timers = active_until;
    while (!stop.load()) {
      // poll window (NBD_OPT_IO_SPIN_US): non-blocking epoll_wait for a while after activity.
      // It takes no lock (timers() runs at most every 500 us meanwhile), so it does not contend
      // with the application threads' sends and stream flushes.
      const int64_t spin = io_spin_us.load(std::memory_order_relaxed);
      const auto t = Clock::now();
      const bool polling = spin > 0 && t < active_until;
      int n = epoll_wait(ep, evs, 64, polling ? 0 : next_timeout_ms());
      if (n > 0 && spin > 0) active_until = Clock::now() + std::chrono::microseconds(spin);
      if (polling && n == 0) {
        if (t - last_timers >= std::chrono::microseconds(500)) {
          timers();
          last_timers = t;
        }
        __builtin_ia32_pause();
        continue;
      }
      if (n < 0) {
        if (errno == EINTR) continue;
        break;
      }
      for (int i = 0; i < n; ++i) {
        uint64_t tok = evs[i].data.u64;
        if (tok == TOK_WAKE) {
          uint64_t v;
          ssize_t r = ::read(evfd, &v, 8);
          (void)r;
        } else if (tok == TOK_CAP0 || tok == TOK_CAP0 + 1) {
          std::lock_guard<std::mutex> lk(cmu);
          drain_locked((int)(tok - TOK_CAP0));
        } else {
          bool is_listener;
          {
            std::lock_guard<std::mutex> lk(mu);
            is_listener = listeners.count(tok) > 0;
          }
          if (is_listener) on_accept(tok);
          else on_peer(tok, evs[i].events);
        }
      }
      timers();
      last_timers = Clock::now();
    }
  }

  // ---------------------------------------------------------------- lifecycle
  int start() {
    ep = epoll_create1(EPOLL_CLOEXEC);
    evfd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (ep < 0 || evfd < 0) return fail(errstr("epoll/eventfd"));
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = TOK_WAKE;
    epoll_ctl(ep, EPOLL_CTL_ADD, evfd, &ev);
    io = std::thread([this] { loop(); });
    return 0;
  }

  int capture_stop_impl() {
    std::lock_guard<std::mutex> lk(cmu);
    for (int k = 0; k < 2; ++k) {
      Capture& c = cap[k];
      if (c.rfd < 0) continue;
      drain_locked(k);
      emit_locked(k);
      ::dup2(c.saved, c.target);
      ::close(c.saved);
      epoll_ctl(ep, EPOLL_CTL_DEL, c.rfd, nullptr);
      ::close(c.rfd);
      c = Capture();
    }
    return 0;
  }

  void shutdown() {
    capture_stop_impl();
    // Give queued output a short chance to leave before the I/O thread stops.
    auto deadline = Clock::now() + std::chrono::milliseconds(200);
    for (;;) {
      bool empty = true;
      {
        std::lock_guard<std::mutex> lk(mu);
        for (auto& kv : peers) {
          std::lock_guard<std::mutex> lk2(kv.second->omu);
          if (!kv.second->outq.empty() && !kv.second->closed) empty = false;
        }
      }
      if (empty || Clock::now() > deadline) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
    stop = true;
    wake();
    if (io.joinable()) io.join();
    std::lock_guard<std::mutex> lk(mu);
    for (auto& kv : peers) {
      std::lock_guard<std::mutex> lk2(kv.second->omu);
      if (!kv.second->closed && kv.second->fd >= 0) ::close(kv.second->fd);
      kv.second->closed = true;
      kv.second->ocv.notify_all();
    }
    peers.clear();
    by_id.clear();
    active.clear();
    for (auto& kv : listeners) {
      ::close(kv.second.fd);
      if (!kv.second.ipc_path.empty()) ::unlink(kv.second.ipc_path.c_str());
    }
    listeners.clear();
    if (ep >= 0) ::close(ep);
    if (evfd >= 0) ::close(evfd);
    ep = evfd = -1;
  }
};

namespace {
struct Guard {
  nbd_socket* s;
  bool ok;
  explicit Guard(nbd_socket* s_) : s(s_) {
    s->users.fetch_add(1);
    ok = !s->closing.load();
  }
  ~Guard() { s->users.fetch_sub(1); }
};
}  // namespace

extern "C" {

int nbd_version(void) { return 10300; }  // 1.3.0
const char* nbd_last_error(void) { return g_err.c_str(); }

nbd_socket* nbd_socket_new(int type) {
  if (type != NBD_ROUTER && type != NBD_DEALER) {
    g_err = "EINVAL: socket type";
    return nullptr;
  }
  auto* s = new nbd_socket(type);
  if (s->start() != 0) {
    delete s;
    return nullptr;
  }
  return s;
}

int nbd_setopt_int(nbd_socket* s, int opt, int64_t v) {
  Guard g(s);
  if (!g.ok) return fail("ECLOSED");
  switch (opt) {
    case NBD_OPT_HEARTBEAT_IVL_MS: s->hb_ivl_ms = (int)v; break;
    case NBD_OPT_HEARTBEAT_TIMEOUT_MS: s->hb_timeout_ms = (int)v; break;
    case NBD_OPT_ROUTER_MANDATORY: s->mandatory = v != 0; break;
    case NBD_OPT_STREAM_FLUSH_US: s->flush_us = v; break;
    case NBD_OPT_STREAM_MAX_BYTES: s->stream_max = (size_t)v; break;
    case NBD_OPT_RECONNECT_IVL_MS: s->reconnect_ivl_ms = (int)std::max<int64_t>(1, v); break;
    case NBD_OPT_SNDHWM_BYTES: s->hwm = (size_t)v; break;
    case NBD_OPT_RECV_SPIN_US: s->recv_spin_us = std::max<int64_t>(0, v); break;
    case NBD_OPT_IO_SPIN_US: s->io_spin_us = std::max<int64_t>(0, v); break;
    default: return fail("EINVAL: option");
  }
  s->wake();
  return 0;
}

int nbd_setopt_bytes(nbd_socket* s, int opt, const void* data, size_t len) {
  Guard g(s);
  if (!g.ok) return fail("ECLOSED");
  std::string v(static_cast<const char*>(data), len);
  std::lock_guard<std::mutex> lk(s->optmu);
  switch (opt) {
    case NBD_OPT_IDENTITY:
      if (len > 255) return fail("EINVAL: identity longer than 255 bytes");
      s->identity = v;
      break;
    case NBD_OPT_TOKEN: s->token = v; break;
    case NBD_OPT_SIGNAL_PREFIX: s->sig_prefix = v; break;
    default: return fail("EINVAL: option");
  }
  return 0;
}

int nbd_bind(nbd_socket* s, const char* endpoint, char* out, size_t outlen) {
  Guard g(s);
  if (!g.ok) return fail("ECLOSED");
  Addr a;
  if (!parse_ep(endpoint, a)) return fail(std::string("EINVAL: bad endpoint ") + endpoint);
  int fd = -1;
  std::string real;
  std::string ipc_path;
  if (a.ipc) {
    fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    sockaddr_un sa{};
    sa.sun_family = AF_UNIX;
    std::strncpy(sa.sun_path, a.path.c_str(), sizeof(sa.sun_path) - 1);
    ::unlink(a.path.c_str());
    if (::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0) {
      int e = errno;
      ::close(fd);
      errno = e;
      return fail(errstr("bind"));
    }
    real = endpoint;
    ipc_path = a.path;
  } else {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_flags = AI_PASSIVE;
    const char* host = (a.host == "*" || a.host.empty()) ? nullptr : a.host.c_str();
    if (host && std::strchr(host, ':')) hints.ai_family = AF_INET6;
    int grc = getaddrinfo(host, a.port.c_str(), &hints, &res);
    if (grc != 0 || !res) return fail(std::string("getaddrinfo: ") + gai_strerror(grc));
    fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (::bind(fd, res->ai_addr, res->ai_addrlen) != 0) {
      int e = errno;
      freeaddrinfo(res);
      ::close(fd);
      errno = e;
      return fail(errstr("bind"));
    }
    freeaddrinfo(res);
    sockaddr_storage ss{};
    socklen_t sl = sizeof(ss);
    getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &sl);
    int port = ss.ss_family == AF_INET ? ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port)
                                       : ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port);
    std::string h = host ? a.host : "0.0.0.0";
    if (h.find(':') != std::string::npos) h = "[" + h + "]";
    real = "tcp://" + h + ":" + std::to_string(port);
  }
  if (::listen(fd, 512) != 0) {
    ::close(fd);
    return fail(errstr("listen"));
  }
  uint64_t tok;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    tok = s->next_tok++;
    Listener l;
    l.fd = fd;
    l.ipc_path = ipc_path;
    s->listeners[tok] = l;
  }
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = tok;
  epoll_ctl(s->ep, EPOLL_CTL_ADD, fd, &ev);
  if (out && outlen) {
    std::strncpy(out, real.c_str(), outlen - 1);
    out[outlen - 1] = 0;
  }
  return 0;
}

int nbd_connect(nbd_socket* s, const char* endpoint) {
  Guard g(s);
  if (!g.ok) return fail("ECLOSED");
  Addr a;
  if (!parse_ep(endpoint, a)) return fail(std::string("EINVAL: bad endpoint ") + endpoint);
  {
    std::lock_guard<std::mutex> lk(s->mu);
    ConnectRec r;
    r.ep = endpoint;
    r.next_try = Clock::now();
    s->connects.push_back(r);
  }
  s->wake();
  return 0;
}

int nbd_send(nbd_socket* s, int nframes, const void* const* ptrs, const size_t* lens) {
  Guard g(s);
  if (!g.ok) return fail("ECLOSED");
  if (s->type == NBD_ROUTER) {
    if (nframes < 2) return fail("EINVAL: ROUTER messages need [identity, frames...]");
    std::string ident(static_cast<const char*>(ptrs[0]), lens[0]);
    return s->route(&ident, nbd_socket::encode(nframes, ptrs, lens, 1), true);
  }
  if (nframes < 1) return fail("EINVAL: empty message");
  return s->route(nullptr, nbd_socket::encode(nframes, ptrs, lens, 0), true);
}

int nbd_send_multi(nbd_socket* s, int nidents, const void* const* iptrs, const size_t* ilens, int nframes,
                   const void* const* ptrs, const size_t* lens, int* status) {
  Guard g(s);
  if (!g.ok) return fail("ECLOSED");
  if (s->type != NBD_ROUTER) return fail("EINVAL: nbd_send_multi needs a ROUTER socket");
  if (nframes < 1) return fail("EINVAL: empty message");
  // encode the frames once, route a copy to every identity (one call fans a cell out to N ranks)
  const std::string body = nbd_socket::encode(nframes, ptrs, lens, 0);
  int failed = 0;
  for (int i = 0; i < nidents; ++i) {
    std::string ident(static_cast<const char*>(iptrs[i]), ilens[i]);
    const int rc = s->route(&ident, std::string(body), true);
    int st = 0;
    if (rc != 0) {
      st = g_err.compare(0, 12, "EHOSTUNREACH") == 0 ? 1 : 2;
      ++failed;
    }
    if (status) status[i] = st;
  }
  return failed;
}

int nbd_recv(nbd_socket* s, int timeout_ms, nbd_msg** out) {
  Guard g(s);
  if (!g.ok) return -1;
  s->spin_for_inbox(timeout_ms);
  std::unique_lock<std::mutex> lk(s->imu);
  auto pred = [s] { return !s->inbox.empty() || s->inbox_closed || s->wake_pending.load(); };
  if (timeout_ms < 0) s->icv.wait(lk, pred);
  // system_clock deadline -> pthread_cond_timedwait (steady_clock would use
  // pthread_cond_clockwait, which older ThreadSanitizer runtimes do not intercept)
  else if (!s->icv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms), pred))
    return 1;
  if (s->inbox.empty()) {
    if (s->inbox_closed) return -1;
    s->wake_pending = false;  // woken by nbd_wake_recv
    return 1;
  }
  Msg* m = s->inbox.front();
  s->inbox.pop_front();
  s->inbox_n.store(s->inbox.size(), std::memory_order_release);
  auto* w = new nbd_msg;
  w->m = std::move(*m);
  delete m;
  *out = w;
  return 0;
}

int nbd_recv_batch(nbd_socket* s, int timeout_ms, void* buf, size_t cap, size_t* used, int max_msgs) {
  Guard g(s);
  if (!g.ok) return -1;
  *used = 0;
  s->spin_for_inbox(timeout_ms);
  std::unique_lock<std::mutex> lk(s->imu);
  auto pred = [s] { return !s->inbox.empty() || s->inbox_closed || s->wake_pending.load(); };
  if (timeout_ms < 0) s->icv.wait(lk, pred);
  else if (!s->icv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms), pred))
    return 0;
  if (s->inbox.empty()) {
    if (s->inbox_closed) return -1;
    s->wake_pending = false;  // woken by nbd_wake_recv
    return 0;
  }
  // serialise queued messages: u32 kind, u32 event, u32 nframes, then (u64 len, bytes) per frame
  char* out = static_cast<char*>(buf);
  size_t pos = 0;
  int n = 0;
  while (!s->inbox.empty() && n < max_msgs) {
    Msg* m = s->inbox.front();
    size_t need = 12;
    for (const auto& f : m->frames) need += 8 + f.size();
    if (pos + need > cap) {
      if (n == 0) {  // the first message alone does not fit: report its size, keep it queued
        *used = need;
        return -2;
      }
      break;
    }
    const uint32_t hdr[3] = {(uint32_t)m->kind, (uint32_t)m->event, (uint32_t)m->frames.size()};
    std::memcpy(out + pos, hdr, 12);
    pos += 12;
    for (const auto& f : m->frames) {
      const uint64_t len = f.size();
      std::memcpy(out + pos, &len, 8);
      pos += 8;
      if (len) std::memcpy(out + pos, f.data(), len);
      pos += len;
    }
    s->inbox.pop_front();
    delete m;
    ++n;
  }
  s->inbox_n.store(s->inbox.size(), std::memory_order_release);
  *used = pos;
  return n;
}

int nbd_wake_recv(nbd_socket* s) {
  Guard g(s);
  if (!g.ok) return fail("ECLOSED");
  {
    std::lock_guard<std::mutex> lk(s->imu);
    s->wake_pending = true;
  }
  s->icv.notify_all();
  return 0;
}

int nbd_msg_kind(const nbd_msg* m) { return m->m.kind; }
int nbd_msg_event(const nbd_msg* m) { return m->m.event; }
int nbd_msg_nframes(const nbd_msg* m) { return (int)m->m.frames.size(); }
int nbd_msg_frames(const nbd_msg* m, const void** ptrs, size_t* lens, int max) {
  int n = (int)std::min<size_t>((size_t)max, m->m.frames.size());
  for (int i = 0; i < n; ++i) {
    ptrs[i] = m->m.frames[(size_t)i].data();
    lens[i] = m->m.frames[(size_t)i].size();
  }
  return n;
}
void nbd_msg_free(nbd_msg* m) { delete m; }

int nbd_peer_count(nbd_socket* s) {
  Guard g(s);
  std::lock_guard<std::mutex> lk(s->mu);
  return (int)s->active.size();
}

int nbd_capture_fds(nbd_socket* s, int mask, int* saved_out, int* saved_err) {
  Guard g(s);
  if (!g.ok) return fail("ECLOSED");
  if (s->type != NBD_DEALER) return fail("EINVAL: capture needs a DEALER socket");
  if (saved_out) *saved_out = -1;
  if (saved_err) *saved_err = -1;
  std::lock_guard<std::mutex> lk(s->cmu);
  for (int k = 0; k < 2; ++k) {
    if (!(mask & (1 << k))) continue;
    Capture& c = s->cap[k];
    if (c.rfd >= 0) continue;
    int target = k + 1;
    int pfd[2];
    if (::pipe2(pfd, O_CLOEXEC) != 0) return fail(errstr("pipe2"));
    ::fcntl(pfd[0], F_SETFL, ::fcntl(pfd[0], F_GETFL) | O_NONBLOCK);
    ::fcntl(pfd[1], F_SETPIPE_SZ, 1 << 20);
    c.saved = ::fcntl(target, F_DUPFD_CLOEXEC, 3);
    ::dup2(pfd[1], target);
    ::close(pfd[1]);
    c.rfd = pfd[0];
    c.target = target;
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = TOK_CAP0 + (uint64_t)k;
    epoll_ctl(s->ep, EPOLL_CTL_ADD, c.rfd, &ev);
    if (k == 0 && saved_out) *saved_out = c.saved;
    if (k == 1 && saved_err) *saved_err = c.saved;
  }
  return 0;
}

int nbd_capture_stop(nbd_socket* s) {
  Guard g(s);
  return s->capture_stop_impl();
}

int nbd_stream_header(nbd_socket* s, int stream, const void* hdr, size_t len) {
  Guard g(s);
  if (!g.ok) return fail("ECLOSED");
  if (stream < 1 || stream > 2) return fail("EINVAL: stream");
  std::lock_guard<std::mutex> lk(s->cmu);
  s->emit_locked(stream - 1);
  s->stream_hdr[stream - 1].assign(static_cast<const char*>(hdr), len);
  return 0;
}

int nbd_stream_flush(nbd_socket* s) {
  Guard g(s);
  if (!g.ok) return fail("ECLOSED");
  std::lock_guard<std::mutex> lk(s->cmu);
  for (int k = 0; k < 2; ++k) {
    s->drain_locked(k);
    s->emit_locked(k);
  }
  return 0;
}

void nbd_close(nbd_socket* s) {
  if (!s) return;
  if (s->closing.exchange(true)) return;
  {
    std::lock_guard<std::mutex> lk(s->imu);
    s->inbox_closed = true;
  }
  s->icv.notify_all();
  // wait for API calls in flight (a blocked nbd_recv returns -1 after the notify above)
  while (s->users.load() > 0) std::this_thread::sleep_for(std::chrono::microseconds(200));
  s->shutdown();
  {
    std::lock_guard<std::mutex> lk(s->imu);
    for (Msg* m : s->inbox) delete m;
    s->inbox.clear();
  }
  // The struct itself stays allocated as a tombstone: a call racing with close (or issued
  // after it) sees closing == true and fails cleanly instead of touching freed memory.
}

}  // extern "C"
