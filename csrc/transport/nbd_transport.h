/*
 * nbd_transport — native control-plane transport for nbdistributed_amd.
 *
 * A small, dependency-free implementation of the ZeroMQ DEALER/ROUTER socket pair speaking
 * ZMTP/3.1 (NULL mechanism) over TCP or Unix-domain sockets, wire-compatible with libzmq.
 *
 * It replaces the reference's pyzmq ROUTER/DEALER pair (reference:
 * src/nbdistributed/communication.py:121-125, worker.py:154-157), which cannot be used here
 * because pyzmq is not importable by the PyTorch-ROCm interpreter, and adds what the
 * reference lacks:
 *   - an epoll I/O thread that runs outside the Python GIL (heartbeats keep flowing while a
 *     worker is busy in a long cell);
 *   - ZMTP/3.1 PING/PONG heartbeats and connect/disconnect events (fail-fast death detection);
 *   - an optional shared-secret token carried as READY metadata (X-Nbd-Token);
 *   - ROUTER "mandatory" routing: sends to an unknown identity fail instead of vanishing;
 *   - native capture of a worker's fd 1/fd 2 into pipes, drained and coalesced (time/size
 *     window) into stream messages by the I/O thread — Python and C-level output share one
 *     ordered path and the main thread never blocks on it;
 *   - "signal on prefix": an inbound message whose first frame starts with a configured prefix
 *     raises SIGINT in the receiving process from the I/O thread (out-of-band interrupt of a
 *     busy worker).
 *
 * Exposed as a C ABI so the same .so serves any Python (ctypes) — the PyTorch workers and a
 * torch-less IPython coordinator alike.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { NBD_ROUTER = 1, NBD_DEALER = 2 };

/* message kinds returned by nbd_recv */
enum { NBD_KIND_MSG = 0, NBD_KIND_EVENT = 1 };

/* event codes (NBD_KIND_EVENT); frame 0 of an event is the peer identity */
enum {
  NBD_EV_CONNECTED = 1,         /* handshake complete */
  NBD_EV_DISCONNECTED = 2,      /* peer closed the connection / connection error */
  NBD_EV_HANDSHAKE_FAILED = 3,  /* bad greeting, incompatible socket type, bad mechanism */
  NBD_EV_HEARTBEAT_TIMEOUT = 4, /* no traffic from the peer within the heartbeat timeout */
  NBD_EV_AUTH_FAILED = 5        /* token mismatch */
};

/* socket options */
enum {
  NBD_OPT_IDENTITY = 1,          /* bytes: routing identity announced in READY (DEALER) */
  NBD_OPT_TOKEN = 2,             /* bytes: shared secret; sent as X-Nbd-Token, checked if set */
  NBD_OPT_HEARTBEAT_IVL_MS = 3,  /* int: PING interval, 0 = off */
  NBD_OPT_HEARTBEAT_TIMEOUT_MS = 4, /* int: drop a peer silent for this long, 0 = off */
  NBD_OPT_ROUTER_MANDATORY = 5,  /* int: ROUTER send to unknown identity fails (EHOSTUNREACH) */
  NBD_OPT_STREAM_FLUSH_US = 6,   /* int: coalescing window for captured output */
  NBD_OPT_STREAM_MAX_BYTES = 7,  /* int: flush captured output once this many bytes are buffered */
  NBD_OPT_SIGNAL_PREFIX = 8,     /* bytes: inbound frame-0 prefix that raises SIGINT */
  NBD_OPT_RECONNECT_IVL_MS = 9,  /* int: DEALER reconnect interval */
  NBD_OPT_SNDHWM_BYTES = 10,     /* int: max queued outbound bytes per peer before send blocks */
  NBD_OPT_RECV_SPIN_US = 11,     /* int: nbd_recv / nbd_recv_batch poll the inbox this long before sleeping */
  NBD_OPT_IO_SPIN_US = 12        /* int: the I/O thread polls its descriptors this long after activity */
};

typedef struct nbd_socket nbd_socket;
typedef struct nbd_msg nbd_msg;

int nbd_version(void);
const char* nbd_last_error(void);

nbd_socket* nbd_socket_new(int type);
int nbd_setopt_int(nbd_socket* s, int opt, int64_t value);
int nbd_setopt_bytes(nbd_socket* s, int opt, const void* data, size_t len);

/* endpoint: "tcp://host:port" (port 0 or * = ephemeral) or "ipc:///path".  The bound endpoint
 * (with the real port) is written to out. */
int nbd_bind(nbd_socket* s, const char* endpoint, char* out, size_t outlen);
int nbd_connect(nbd_socket* s, const char* endpoint);

/* Send one multipart message. ROUTER: frame 0 is the destination identity.
 * Returns 0, or -1 (errno-style code in nbd_last_error). */
int nbd_send(nbd_socket* s, int nframes, const void* const* ptrs, const size_t* lens);

/* ROUTER: send the same multipart body (frames, no identity) to each of nidents identities,
 * encoding it once.  status[i] = 0 sent, 1 no such peer (EHOSTUNREACH, mandatory routing),
 * 2 other error.  Returns the number of failed identities, or -1 if the call itself failed. */
int nbd_send_multi(nbd_socket* s, int nidents, const void* const* iptrs, const size_t* ilens, int nframes,
                   const void* const* ptrs, const size_t* lens, int* status);

/* Wait up to timeout_ms (-1 = forever) for a message or event.
 * Returns 0 with *out set, 1 on timeout, -1 if the socket is closed. */
int nbd_recv(nbd_socket* s, int timeout_ms, nbd_msg** out);
/* Drain up to max_msgs queued messages (waiting up to timeout_ms, -1 = forever, for the first)
 * into buf, serialised as: u32 kind, u32 event, u32 nframes, then per frame u64 length + bytes
 * (native endianness).  Returns the number of messages (0 on timeout), -1 if the socket is
 * closed, -2 if the first queued message needs more than cap bytes (*used = the size needed;
 * it stays queued).  One call replaces recv + 5 accessor calls + free per message. */
int nbd_recv_batch(nbd_socket* s, int timeout_ms, void* buf, size_t cap, size_t* used, int max_msgs);
/* Make the nbd_recv / nbd_recv_batch call blocked right now — or, if none is, the next one that
 * finds the inbox empty — return as on a timeout (1 / 0).  Sticky until consumed, so a wake
 * cannot be lost to a receiver that is just about to block. */
int nbd_wake_recv(nbd_socket* s);
int nbd_msg_kind(const nbd_msg* m);
int nbd_msg_event(const nbd_msg* m);
int nbd_msg_nframes(const nbd_msg* m);
int nbd_msg_frames(const nbd_msg* m, const void** ptrs, size_t* lens, int max);
void nbd_msg_free(nbd_msg* m);

/* number of peers that completed the handshake */
int nbd_peer_count(nbd_socket* s);

/* Output capture (DEALER only).  mask bit0 = fd 1, bit1 = fd 2.  The original descriptors are
 * dup'ed and returned through saved_out / saved_err (-1 if not captured).  Captured bytes are
 * sent as two-frame messages [header(stream), bytes] where header(stream) is the template set
 * by nbd_stream_header (stream 1 = stdout, 2 = stderr). */
int nbd_capture_fds(nbd_socket* s, int mask, int* saved_out, int* saved_err);
int nbd_capture_stop(nbd_socket* s);
int nbd_stream_header(nbd_socket* s, int stream, const void* hdr, size_t len);
/* Drain the capture pipes and send everything buffered, in order, before returning. */
int nbd_stream_flush(nbd_socket* s);

void nbd_close(nbd_socket* s);

#ifdef __cplusplus
}
#endif
