/*
 * kmws_gpu.h -- C ABI of the MI355X (gfx950) WebSocket frame codec.
 *
 * Drop-in boundary for kuma's RFC 6455 codec (reference: src/ws/WSHandler.h:32-91,
 * used by WebSocket::Impl, src/ws/WebSocketImpl.cpp).  Plain C: fixed-width
 * integers, raw pointers and sizes; a HIP stream is passed as `void*`
 * (a hipStream_t, NULL = the default stream).  Every function returns a
 * kmws_status (0 = OK, negative = kuma KMError value, include/kmdefs.h:61-86)
 * unless noted; codec results use kuma's WSError numbering (wsdefs.h:56-67).
 *
 * Three families:
 *  - host codec entries (kmws_encode_header, kmws_decoder_*): the per-connection,
 *    byte-stream state machine that kuma runs on its event-loop thread.  The
 *    decoder parses headers on the host; payload unmasking is done by the GPU
 *    kernels below (batched per feed call).  See DESIGN.md "Boundary".
 *  - loop-level host batches: kmws_rx_batch_* (receive: one GPU batch per
 *    event-loop iteration across reads and connections), kmws_tx_batch_*
 *    (send: one GPU mask launch for every send of an iteration),
 *    kmws_mask_host_chain and kmws_pipeline_* (host-resident frame batches);
 *    synchronous, pinned staging or zero-copy on caller-pinned memory.
 *  - device batch entries (kmws_*_batch, kmws_unpack_headers,
 *    kmws_gather_unmask): stream-ordered, no host sync, no allocation; all
 *    pointers are device pointers; workspace is caller-owned.  The one set-up
 *    call, kmws_unmask_autotune, synchronizes.
 *
 * Bench / test support (arenas, synthetic batches, the device checker) lives
 * in include/kmws_bench.h, outside this boundary.
 */
#ifndef KMWS_GPU_H
#define KMWS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes: kuma KMError values (include/kmdefs.h:61-86) ---- */
typedef int kmws_status;
#define KMWS_OK                    0
#define KMWS_ERR_FAILED           (-1)   /* KMError::FAILED (HIP runtime error) */
#define KMWS_ERR_TIMEOUT          (-6)   /* KMError::TIMEOUT: a host job the device neither finished nor
                                            gave up in time; the device may still write its buffer */
#define KMWS_ERR_INVALID_STATE    (-7)   /* KMError::INVALID_STATE */
#define KMWS_ERR_INVALID_PARAM    (-8)   /* KMError::INVALID_PARAM */
#define KMWS_ERR_BUFFER_TOO_SMALL (-17)  /* KMError::BUFFER_TOO_SMALL */
#define KMWS_ERR_BUFFER_TOO_LONG  (-18)  /* KMError::BUFFER_TOO_LONG (a send of more than 128 segments) */
#define KMWS_ERR_NOT_SUPPORTED    (-19)  /* KMError::NOT_SUPPORTED (no gfx950 device) */

/* The resident worker's job limits (kmws_resident.hip): the masked payloads of
 * one call or one submitted generation, at most KMWS_RESIDENT_MAX_PAYLOADS of
 * them and KMWS_RESIDENT_MAX_BYTES bytes, run on the calling thread's slot of
 * the device's resident grid without a kernel launch; larger jobs, and a job
 * posted while the thread's previous one still runs, launch instead.  The
 * loop helpers (include/kmws_wshandler.hpp) size their generations to fit. */
#define KMWS_RESIDENT_MAX_PAYLOADS 128
#define KMWS_RESIDENT_MAX_BYTES (256u << 10)

/* ---- device selection (SURVEY 8 e): which GPU a loop thread's objects use ----
 * kuma runs a pool of event-loop threads (test/client/main.cpp:20,
 * test/server/main.cpp:22) and every connection's bytes arrive on its loop
 * thread (TcpConnection.cpp:229).  Every `device` argument below also accepts
 * KMWS_DEVICE_AUTO: the calling thread's device, kmws_thread_device() -- the
 * one kmws_set_thread_device pinned, else chosen once for the thread by the
 * process's policy: NUMA (default: round robin over the GPUs on the NUMA node
 * of the CPU the thread runs on, over all GPUs when that node has none),
 * ROUND_ROBIN (over all GPUs, in the order threads first ask), FIRST (device
 * 0).  So each loop thread's payloads cross its own GPU's PCIe link into its
 * own pinned staging; host DRAM is what the threads still share.  A thread's
 * device does not change once chosen.  The library reads no environment. */
#define KMWS_DEVICE_AUTO (-1)
enum kmws_device_policy { KMWS_DEVICE_POLICY_NUMA = 0, KMWS_DEVICE_POLICY_ROUND_ROBIN = 1,
                          KMWS_DEVICE_POLICY_FIRST = 2 };
kmws_status kmws_set_device_policy(int policy);  /* process-wide; threads that chose keep their device */
/* Pins the calling thread to `device` (KMWS_DEVICE_AUTO: back to the policy for
 * objects created later).  KMWS_ERR_NOT_SUPPORTED: no such gfx950 device. */
kmws_status kmws_set_thread_device(int device);
/* The calling thread's device (>= 0), or KMWS_ERR_NOT_SUPPORTED without a
 * gfx950 device. */
int         kmws_thread_device(void);
/* Claims the calling thread's slot of `device`'s resident grid now (the
 * synchronous entries and batch submits otherwise claim it at their first
 * job) and registers the thread-exit hook that gives it back -- after every
 * thread_local object constructed before this call returned, i.e. after a
 * thread_local loop object whose constructor calls it (kmws::RxLoop, TxLoop),
 * so that object's destructor still flushes on the slot.  A job asked for
 * after the hook ran launches instead.  Returns the slot, or negative: no
 * slot free (jobs launch), the worker is off for this thread, or no device. */
int         kmws_thread_attach(int device);

/* ---- codec results: WSError (src/ws/wsdefs.h:56-67) ---- */
enum kmws_ws_error {
    KMWS_WS_NOERR = 0, KMWS_WS_NEED_MORE_DATA = 1, KMWS_WS_HANDSHAKE = 2,
    KMWS_WS_INVALID_PARAM = 3, KMWS_WS_INVALID_STATE = 4, KMWS_WS_INVALID_FRAME = 5,
    KMWS_WS_INVALID_LENGTH = 6, KMWS_WS_PROTOCOL_ERROR = 7, KMWS_WS_CLOSED = 8,
    KMWS_WS_DESTROYED = 9
};

/* WSMode (wsdefs.h:69-72) */
enum kmws_mode { KMWS_MODE_CLIENT = 0, KMWS_MODE_SERVER = 1 };

/* WSOpcode (wsdefs.h:47-54) */
enum kmws_opcode { KMWS_OP_CONTINUE = 0, KMWS_OP_TEXT = 1, KMWS_OP_BINARY = 2,
                   KMWS_OP_CLOSE = 8, KMWS_OP_PING = 9, KMWS_OP_PONG = 10 };

#define KMWS_MASK_KEY_SIZE   4          /* WS_MASK_KEY_SIZE, wsdefs.h:36 */
#define KMWS_MAX_HEADER_SIZE 14         /* WS_MAX_HEADER_SIZE, wsdefs.h:37 */
#define KMWS_MAX_FRAME_DATA_LENGTH (10u * 1024u * 1024u)  /* WSHandler.cpp:110 */

/* FrameHeader (wsdefs.h:74-88) with the bitfields widened to bytes. */
typedef struct kmws_frame_hdr {
    uint8_t  fin, rsv1, rsv2, rsv3, opcode, mask, plen, reserved;
    uint64_t xpl64;                      /* union xpl: xpl16 = low 16 bits */
    uint8_t  maskey[KMWS_MASK_KEY_SIZE]; /* wire order */
    uint32_t length;
} kmws_frame_hdr;

/* Frame descriptor in HBM (16 B): payload at base+off, len bytes, key = the
 * 4 wire key bytes read as a little-endian u32 (== *(uint32_t*)hdr.maskey,
 * WebSocketImpl.cpp:386). */
typedef struct kmws_desc {
    uint64_t off;
    uint32_t len;
    uint32_t key;
} kmws_desc;

/* Per-frame flags for the pack kernels: bits 0-7 = header byte 0
 * (fin<<7 | rsv1<<6 | rsv2<<5 | rsv3<<4 | opcode), bit 8 = mask. */
#define KMWS_FLAG_MASK 0x100u
static inline uint16_t kmws_make_flags(int fin, int rsv1, int rsv2, int rsv3, int opcode, int mask)
{
    return (uint16_t)((fin ? 0x80 : 0) | (rsv1 ? 0x40 : 0) | (rsv2 ? 0x20 : 0) |
                      (rsv3 ? 0x10 : 0) | (opcode & 0x0F) | (mask ? KMWS_FLAG_MASK : 0));
}

/* ======================= host codec entries ======================= */

/* WSHandler::encodeFrameHeader (WSHandler.cpp:46-106).  Returns the header
 * length (2, 4 or 10, +4 when masked); out must hold 14 bytes. */
int kmws_encode_header(const kmws_frame_hdr* hdr, uint8_t out[KMWS_MAX_HEADER_SIZE]);

/* Length of the header kmws_encode_header would write (2/4/10 + 4*mask). */
int kmws_header_size(uint32_t length, int mask);

/* ---- streaming decoder: WSHandler (WSHandler.h:32-91) ---- */
typedef struct kmws_decoder kmws_decoder;

/* Frame callback: WSHandler::FrameCallback (WSHandler.h:35).  The payload
 * view is valid only during the call (WSHandler.cpp:285).  Return nonzero if
 * the callback destroyed the owner; the decoder then returns
 * KMWS_WS_DESTROYED without touching itself (DESTROY_DETECTOR, :284-287). */
typedef int (*kmws_frame_cb)(const kmws_frame_hdr* hdr, uint8_t* payload, size_t len, void* user);

/* mode: kmws_mode.  device: HIP device used for payload unmasking. */
kmws_decoder* kmws_decoder_create(int mode, int device);
void          kmws_decoder_destroy(kmws_decoder* dec);
void          kmws_decoder_set_mode(kmws_decoder* dec, int mode);   /* WSHandler::setMode */
void          kmws_decoder_reset(kmws_decoder* dec);                /* WSHandler::reset, :324-327 */

/* WSHandler::handleData (WSHandler.cpp:41-44 -> decodeFrame :108-280).
 * Same return values and callback sequence; masked payloads are unmasked by
 * the GPU (one batched launch per call) and, as in kuma, in place in `data`
 * when a frame lies wholly inside it.  If `data` is pinned host memory the
 * kernel unmasks it there directly (zero-copy, rewriting the 16-B hulls of
 * those payloads); otherwise payloads go through a pinned staging copy.
 * Returns a kmws_ws_error value, or a negative kmws_status if the GPU step
 * failed. */
int kmws_decoder_feed(kmws_decoder* dec, uint8_t* data, size_t len, kmws_frame_cb cb, void* user);

/* In-place contract of kmws_decoder_feed for a PAGEABLE chunk (on by default).
 * Off: a masked payload lying in the chunk is delivered as a view of its
 * unmasked pinned staging copy and the chunk keeps its masked bytes -- one
 * host copy fewer per read.  kuma cannot tell the difference: its read buffer
 * is not touched after handleData returns (TcpConnection.cpp:229-238) and the
 * frame callback only sees the view (WSHandler.cpp:285).  Pinned chunks are
 * always unmasked in place (zero-copy). */
void kmws_decoder_set_in_place(kmws_decoder* dec, int on);

/* WSHandler::handleDataMask(key, KMBuffer&) (WSHandler.cpp:312-322) and, with
 * nseg == 1, handleDataMask(key, data, len) (:303-310) for HOST buffers: the
 * segments of a chain are masked in place with the key phase continuing
 * across segments.  Runs on the GPU (gathered into pinned staging, one
 * unmask launch, scattered back); synchronous; per-thread staging. */
kmws_status kmws_mask_host_chain(const uint8_t key[KMWS_MASK_KEY_SIZE], uint8_t* const* segs, const size_t* lens,
                                 size_t nseg, int device);

/* ---- deferred delivery: one GPU batch per event-loop iteration (SURVEY f-1) ----
 * kuma calls handleData once per 64 KiB socket read per connection; a GPU
 * round trip per call costs more than the scalar unmask it replaces.  A loop
 * thread instead feeds every read of every connection with
 * kmws_decoder_feed_deferred (headers parsed and validated immediately, same
 * return values as kmws_decoder_feed; payloads copied into the batch) and
 * once per iteration either calls kmws_rx_batch_flush -- one GPU unmask over
 * all staged payloads, then every deferred callback in feed order -- or,
 * asynchronously, kmws_rx_batch_submit (enqueues the unmask of the iteration's
 * frames and returns at once) and kmws_rx_batch_poll at the next iterations
 * (delivers the callbacks of every submitted generation whose unmask has
 * finished, in submit order; wait != 0: all of them), so the GPU round trip
 * overlaps the loop's socket reads (the EventLoop::post pattern,
 * kmapi.h:204-210).  Payload views point into the batch (or the attached
 * ring) and are valid during the callback; the caller's chunk is not
 * modified.  A callback returning nonzero ("destroyed") drops every other frame
 * of that decoder still held by the batch: the rest of the generation, later
 * generations in flight and the generation being fed.  Destroy a decoder only after its
 * frames were delivered or after kmws_rx_batch_discard (which also covers
 * submitted generations).  Do not mix kmws_decoder_feed and deferred feeds on
 * one decoder while its frames are pending. */
typedef struct kmws_rx_batch kmws_rx_batch;
kmws_rx_batch* kmws_rx_batch_create(int device);      /* NULL without a gfx950 device */
void           kmws_rx_batch_destroy(kmws_rx_batch* b);
int            kmws_decoder_feed_deferred(kmws_decoder* dec, kmws_rx_batch* b, const uint8_t* data, size_t len,
                                          kmws_frame_cb cb, void* user);
int            kmws_rx_batch_flush(kmws_rx_batch* b);  /* frames delivered, or negative status */
int            kmws_rx_batch_submit(kmws_rx_batch* b); /* frames submitted (0: none), or negative status */
int            kmws_rx_batch_poll(kmws_rx_batch* b, int wait);  /* frames delivered, or negative status */
int            kmws_rx_batch_pending(const kmws_rx_batch* b);   /* frames fed, not yet submitted */
uint64_t       kmws_rx_batch_pending_bytes(const kmws_rx_batch* b);  /* their masked payload bytes */
int            kmws_rx_batch_inflight(const kmws_rx_batch* b);  /* generations submitted, not yet delivered */
/* Optional pinned receive ring (hipHostMalloc / hipHostRegister, e.g.
 * kmws_host_alloc) that the loop reads sockets into: chunks fed from inside it
 * are not copied -- their masked payloads are unmasked in place there
 * (zero-copy), and the callback views point into the ring.  The ring bytes of a
 * frame must stay unmodified until the frame is delivered.  Only while the
 * batch holds no frames; NULL detaches. */
kmws_status    kmws_rx_batch_attach_ring(kmws_rx_batch* b, uint8_t* ring, size_t bytes);
void           kmws_rx_batch_discard(kmws_rx_batch* b, const kmws_decoder* dec);

/* ---- batched send path: one GPU batch per event-loop iteration (SURVEY f-2) ----
 * WebSocket::Impl::sendWsFrame (WebSocketImpl.cpp:381-436) masks the caller's
 * payload in place and packs the header, once per send.  A loop thread
 * instead queues every send of the iteration with kmws_tx_batch_add -- the
 * header is packed at once into hdr_out (length = (uint32_t) payload bytes,
 * :390/:415, then encodeFrameHeader) and the payload segments are queued for
 * masking with hdr->maskey when hdr->mask is set and the payload is not empty
 * (kuma's client mode: mask = 1 and a fresh key per frame, :386/:411; keys are
 * inputs here) -- and masks every queued payload in place with one GPU launch,
 * key phase continuing across a frame's segments: kmws_tx_batch_flush
 * (synchronous), or kmws_tx_batch_submit (returns a ticket at once) and
 * kmws_tx_batch_poll(ticket) (1 once every generation up to the ticket is
 * masked and back in the caller's buffers, 0 while in flight; wait != 0
 * blocks), so the loop fills and submits the next iteration's sends while
 * this one's masks run.  The segments must stay valid and unmodified until
 * their generation completed; the iovec list for the socket is then [hdr_out,
 * segments...] as in :419-431.  A send with more than 128 non-empty segments
 * returns KMWS_ERR_BUFFER_TOO_LONG, and -- as in kuma, which masks before
 * counting iovecs -- its payload is still masked.  Payloads over 4 GiB - 1
 * are refused (KMWS_ERR_INVALID_PARAM). */
typedef struct kmws_tx_batch kmws_tx_batch;
kmws_tx_batch* kmws_tx_batch_create(int device);      /* NULL without a gfx950 device */
void           kmws_tx_batch_destroy(kmws_tx_batch* b);
/* Returns the header length (2..14) or a negative kmws_status. */
int            kmws_tx_batch_add(kmws_tx_batch* b, const kmws_frame_hdr* hdr, uint8_t* const* segs,
                                 const size_t* lens, size_t nseg, uint8_t hdr_out[KMWS_MAX_HEADER_SIZE]);
/* Masks every queued payload (one launch, synchronous); returns the number of
 * frames masked, or a negative kmws_status.  The batch is empty afterwards. */
int64_t        kmws_tx_batch_flush(kmws_tx_batch* b);
/* Enqueues the mask of every queued payload; returns its ticket (> 0), 0 if
 * nothing was queued, or a negative kmws_status. */
int64_t        kmws_tx_batch_submit(kmws_tx_batch* b);
int            kmws_tx_batch_poll(kmws_tx_batch* b, int64_t ticket, int wait);
int            kmws_tx_batch_pending(const kmws_tx_batch* b);
/* Optional pinned send ring (hipHostMalloc / hipHostRegister) the loop builds
 * its outgoing payloads in: segments inside it are masked in place there
 * (zero-copy, one launch), the others go through pinned staging.  Only while
 * no sends are queued or in flight (KMWS_ERR_INVALID_STATE otherwise); NULL
 * detaches. */
kmws_status    kmws_tx_batch_attach_ring(kmws_tx_batch* b, uint8_t* ring, size_t ring_bytes);

/* ======================= device batch entries ======================= */

/* Number of HIP devices of arch gfx950 visible (0 => device entries return
 * KMWS_ERR_NOT_SUPPORTED).  Never falls back to the CPU. */
int kmws_device_count(void);

/* Workspace bytes needed by kmws_unmask_batch for `span` bytes of payload
 * address space (tile map + status word). */
size_t kmws_unmask_workspace_size(uint64_t span);

/* Batched in-place unmask (replaces WSHandler::handleDataMask, WSHandler.cpp:
 * 291-310, for a whole batch).  Frame i's bytes base[off .. off+len) are XORed
 * with key byte (j % 4) for payload position j.  Preconditions: descs sorted
 * by off, non-overlapping, off+len <= span; base 16-byte aligned.  The kernel
 * rewrites whole 16-byte words of each frame's aligned hull (bytes outside a
 * payload keep their value); nothing may write those hull bytes concurrently.
 * A precondition violation sets the workspace status word (kmws_read_status)
 * and leaves the payload untouched. */
kmws_status kmws_unmask_batch(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                              void* workspace, size_t workspace_bytes, void* stream);

/* kmws_unmask_batch in two stream-ordered halves: `plan` validates the
 * descriptors and builds the tile map in the workspace; `apply` runs the
 * unmask kernel with the default schedule.  A plan stays valid for the same
 * (descs, n, span). */
kmws_status kmws_unmask_plan(uint64_t span, const kmws_desc* descs, uint32_t n, void* workspace,
                             size_t workspace_bytes, void* stream);
kmws_status kmws_unmask_apply(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                              const void* workspace, size_t workspace_bytes, void* stream);

/* Unmask schedules.  The apply grid is one block per 16 KiB tile; a schedule
 * says which tiles the resident blocks stream at once and how the payload is
 * stored.  Placement kind (low byte): */
#define KMWS_SCHED_GROUPED_RUNS 0   /* XCDs in 2 groups, runs of 16 tiles in each group's half
                                       (the default below a mean frame region of 16 KiB) */
#define KMWS_SCHED_IN_ORDER     1   /* tile = block */
#define KMWS_SCHED_SPLIT2       2   /* blocks dealt over 2 far-apart parts of the span */
#define KMWS_SCHED_SPLIT8       3   /* ... over 8 parts */
#define KMWS_SCHED_XCD_RUNS     4   /* runs of 16 tiles per XCD */
#define KMWS_SCHED_SPLIT4       5   /* ... over 4 parts (the default from a 16 KiB mean region) */
/* Store policy of the payload: non-temporal by default (neither bit, or
 * KMWS_SCHED_NT_STORES); KMWS_SCHED_TEMPORAL_STORES keeps the lines in L2
 * (written back on eviction) -- slower on plain allocations of every layout
 * measured, a candidate the autotune times.  At most one bit. */
#define KMWS_SCHED_NT_STORES       (1 << 29)
#define KMWS_SCHED_TEMPORAL_STORES (1 << 30)

/* kmws_unmask_apply with an explicit schedule (schedule < 0: the default,
 * kmws_unmask_default_schedule).  The library keeps no schedule state: a
 * schedule belongs to the caller's plan of one batch (e.g. the code
 * kmws_unmask_autotune returned for it) and is passed on every apply, like the
 * descriptors.  An invalid code returns KMWS_ERR_INVALID_PARAM. */
kmws_status kmws_unmask_apply_sched(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                                    const void* workspace, size_t workspace_bytes, int schedule, void* stream);

/* The schedule kmws_unmask_apply / kmws_unmask_batch use: split 4 from a mean
 * frame region of 16 KiB (span / n), grouped XCD runs below; non-temporal
 * stores. */
int kmws_unmask_default_schedule(uint64_t span, uint32_t n);

/* Optional one-time tuning of ONE batch (like a cuDNN benchmark pass): runs
 * every placement kind with both store policies twice on this batch (the XOR
 * applied twice leaves the payload unchanged), times them with events on
 * `stream` (synchronizes) and returns the fastest schedule code (or a negative
 * status) for the caller to pass to kmws_unmask_apply_sched.  Nothing is
 * recorded: the next batch, on any workspace, gets the default unless its
 * caller passes a schedule. */
int kmws_unmask_autotune(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n, void* workspace,
                         size_t workspace_bytes, void* stream);

/* Read (synchronously) the status word of a workspace after a batch call, a
 * bit set: 0 = OK, 1 = descriptor precondition violated (or the output would
 * exceed dst_cap), 2 = header error seen, 4 = a scan timed out waiting for a
 * predecessor tile's state (kmws_pack_headers, and kmws_encode_batch /
 * kmws_gather_unmask in their chunk form: never seen with in-order workgroup
 * dispatch).  The offsets those calls write (wire_off, dst_off) are valid
 * only when the status is 0; with bit 1 or 4 set nothing is stored in dst. */
kmws_status kmws_read_status(const void* workspace, uint32_t* status_out, void* stream);

/* ---- batched header pack / unpack (device) ---- */

/* Workspace bytes for kmws_encode_batch / kmws_gather_unmask with n frames
 * and an output capacity of dst_cap bytes.  The copy form follows dst_cap / n
 * (below 16 KiB per frame: 4 KiB output chunks, one wave each, 8 B of
 * workspace per chunk; from it: per-frame edge words and 32 B per 4 KiB
 * output unit), so size the workspace with the dst_cap the call will pass. */
size_t kmws_copy_workspace_size(uint32_t n, uint64_t dst_cap);

/* Batched frame encode: for frame i, WSHandler::encodeFrameHeader
 * (WSHandler.cpp:46-106) of {flags[i], len, key} followed by the payload
 * src[descs[i].off .. +len) masked with key when flags[i] & KMWS_FLAG_MASK
 * (WebSocketImpl.cpp:381-404), all frames back to back in dst.  wire_off
 * (n+1 entries, device) receives each frame's header offset and, in
 * wire_off[n], the total wire size.  If the total exceeds dst_cap nothing is
 * written and the workspace status word is set.  wire_off and dst are valid
 * only when the status (kmws_read_status) is 0 afterwards.  src and dst 16-B
 * aligned; source payloads may overlap or sit anywhere in src. */
kmws_status kmws_encode_batch(const uint8_t* src, const kmws_desc* descs, const uint16_t* flags, uint32_t n,
                              uint8_t* dst, uint64_t dst_cap, uint64_t* wire_off, void* workspace,
                              size_t workspace_bytes, void* stream);

/* Workspace bytes for kmws_pack_headers with n frames. */
size_t kmws_pack_headers_workspace_size(uint32_t n);

/* Batched header pack only -- the device form of kuma's send iovec
 * {header, payload} (WebSocketImpl.cpp:381-404, :419-431): frame i's header,
 * WSHandler::encodeFrameHeader (WSHandler.cpp:46-106) of {flags[i],
 * descs[i].len, descs[i].key}, is written to the 16-byte slot hdr + 16 i (its
 * hdr_len[i] = 2..14 bytes first, the rest of the slot zero).  The payloads are
 * not touched: mask them in place with kmws_unmask_batch (XOR is its own
 * inverse), as sendWsFrame masks the caller's buffer (:388), on descriptors
 * whose key is 0 for every frame whose flags clear KMWS_FLAG_MASK (the header
 * then says unmasked; a nonzero key there would still be applied).  wire_off
 * (n+1 entries, may be NULL) receives the offsets the frames would have back
 * to back on the wire (exclusive scan of header + payload bytes) and the total
 * in wire_off[n]; it needs the workspace (a status word and one 8-byte scan
 * state per 2048 frames, cleared by the call; one pass over the descriptors).
 * wire_off is valid only when the workspace status (kmws_read_status) is 0
 * afterwards.  hdr 16-B aligned. */
kmws_status kmws_pack_headers(const kmws_desc* descs, const uint16_t* flags, uint32_t n, uint8_t* hdr,
                              uint8_t* hdr_len, uint64_t* wire_off, void* workspace, size_t workspace_bytes,
                              void* stream);

/* Workspace bytes for kmws_unpack_headers. */
size_t kmws_unpack_workspace_size(void);

/* Descriptor-indexed header unpack + validation, one frame per hdr_off entry
 * (offsets ascending, each frame ending by the next header): the HDR1..MASKEY
 * rules of WSHandler::decodeFrame (WSHandler.cpp:118-234) for `mode`,
 * including the 127-class length quirk.  Per frame: out_desc = {payload
 * offset in wire, len, key (0 if unmasked)}, out_flags = header byte 0 |
 * mask << 8 (may be NULL), out_err = WSError (may be NULL): 1 truncated,
 * 6 bad length, 7 protocol error, 5 frame overruns the next header.  Error
 * frames get len 0.  Any error sets status bit 2. */
kmws_status kmws_unpack_headers(const uint8_t* wire, uint64_t wire_len, const uint64_t* hdr_off, uint32_t n,
                                int mode, kmws_desc* out_desc, uint16_t* out_flags, uint8_t* out_err,
                                void* workspace, size_t workspace_bytes, void* stream);

/* kmws_unpack_headers and kmws_unmask_batch fused: the descriptor-indexed
 * decode in place, as kuma unmasks in the caller's buffer (WSHandler.cpp:
 * 247-260).  One kernel parses every header (the kmws_unpack_headers rules and
 * outputs) and writes the unmask plan -- frame i's region is [hdr_off[i],
 * hdr_off[i+1]) -- then the unmask kernel runs on the wire in place with
 * `schedule` (< 0: the default).  workspace: kmws_unmask_workspace_size(wire_len);
 * wire 16-byte aligned.  A header error sets out_err and status bit 2 and
 * leaves that frame masked (len 0), the others are unmasked; offsets out of
 * order or past wire_len set status bit 1 and nothing is unmasked. */
kmws_status kmws_unpack_unmask(uint8_t* wire, uint64_t wire_len, const uint64_t* hdr_off, uint32_t n, int mode,
                               kmws_desc* out_desc, uint16_t* out_flags, uint8_t* out_err, void* workspace,
                               size_t workspace_bytes, int schedule, void* stream);

/* Out-of-place unmask: frame i's payload src[descs[i].off .. +len) XOR its key
 * is written densely to dst at dst_off[i] (exclusive scan of len; n+1
 * entries, dst_off[n] = total).  Nothing is written if total > dst_cap.
 * dst_off and dst are valid only when the workspace status is 0 afterwards. */
kmws_status kmws_gather_unmask(const uint8_t* src, const kmws_desc* descs, uint32_t n, uint8_t* dst,
                               uint64_t dst_cap, uint64_t* dst_off, void* workspace, size_t workspace_bytes,
                               void* stream);

/* kmws_unpack_headers and kmws_gather_unmask fused: the header parse runs
 * inside the gather's first (scan) kernel, which writes out_desc / out_flags /
 * out_err exactly as kmws_unpack_headers does; the payloads are then gathered
 * densely into dst as kmws_gather_unmask does (error frames: len 0).
 * workspace: kmws_copy_workspace_size(n, dst_cap); wire and dst 16-byte
 * aligned.  Status bit 2: a header error was seen. */
kmws_status kmws_unpack_gather(const uint8_t* wire, uint64_t wire_len, const uint64_t* hdr_off, uint32_t n, int mode,
                               kmws_desc* out_desc, uint16_t* out_flags, uint8_t* out_err, uint8_t* dst,
                               uint64_t dst_cap, uint64_t* dst_off, void* workspace, size_t workspace_bytes,
                               void* stream);

/* Host: walk the header chain of a wire image (WSHandler.cpp:108-280 state
 * order, reading only header bytes and skipping payloads) and record each
 * header offset.  Stops after `cap` frames, after a frame that is truncated
 * or has an invalid length (recorded, so kmws_unpack_headers reports it), or
 * after a CLOSE frame (the reference stops parsing there, :265-268).
 * *consumed = bytes covered by the recorded complete frames. */
kmws_status kmws_find_headers(const uint8_t* wire, uint64_t len, uint64_t* hdr_off, uint32_t cap,
                              uint32_t* n_out, uint64_t* consumed);

/* Device: the same header-chain walk as kmws_find_headers, one lane per
 * stream, for many streams at once (boundary discovery is serial within a
 * stream -- frame k+1 starts where frame k's header says -- so a batch gets its
 * parallelism from connections; SURVEY 8 "hard parts").  Stream s is
 * wire[stream_off[s] .. stream_off[s+1]) (stream_off: n_streams+1 ascending
 * entries, stream_off[n_streams] <= wire_len; a stream reaching past wire_len
 * is cut there).  Its header offsets (absolute,
 * into wire) go to hdr_off[s * cap .. s * cap + n_out[s]); consumed[s] (may be
 * NULL) = bytes of stream s covered by its complete frames.  Stopping rules as
 * kmws_find_headers: cap frames, a truncated frame or invalid length (recorded),
 * or after a CLOSE frame.  All pointers device memory. */
kmws_status kmws_find_headers_streams(const uint8_t* wire, uint64_t wire_len, const uint64_t* stream_off,
                                      uint32_t n_streams, uint64_t* hdr_off, uint32_t cap, uint32_t* n_out,
                                      uint64_t* consumed, void* stream);

/* ---- host-resident batches: pinned H2D -> kernel -> D2H pipeline ---- */
typedef struct kmws_pipeline kmws_pipeline;

/* depth slots (streams) of chunk_bytes device buffer each; chunks are cut on
 * frame boundaries with at most max_frames_per_chunk frames. */
kmws_pipeline* kmws_pipeline_create(int device, uint64_t chunk_bytes, uint32_t max_frames_per_chunk, int depth);
void           kmws_pipeline_destroy(kmws_pipeline* p);

/* Transfer mode: AUTO = chunked SDMA copies through device slots (H2D, kernel
 * and D2H on three streams, so both DMA directions run at once), except for a
 * pinned host_base (hipHostMalloc / hipHostRegister) spanning less than two
 * chunks, which gets one zero-copy launch (the kernel reads and writes host
 * memory over PCIe); COPY forces the chunked SDMA path; ZEROCOPY requires
 * pinned memory.  At most 3 slots are used at once whatever the depth. */
enum kmws_xfer { KMWS_XFER_AUTO = 0, KMWS_XFER_COPY = 1, KMWS_XFER_ZEROCOPY = 2 };
kmws_status kmws_pipeline_set_transfer(kmws_pipeline* p, int mode);

/* In-place unmask of frames that live in HOST memory (descs on the host,
 * offsets relative to host_base, sorted, within span).  Synchronous: returns
 * when every byte is back in host_base.  Only the frames' extents are written
 * back by the copy path; the zero-copy path rewrites their 16-B hulls.
 * Every descriptor is checked before anything is queued: unsorted, overlapping
 * or out-of-span frames return KMWS_ERR_INVALID_PARAM, a frame whose 16-B hull
 * exceeds chunk_bytes KMWS_ERR_BUFFER_TOO_SMALL, with host_base untouched; a
 * HIP failure mid-batch drains every queued copy before returning. */
kmws_status kmws_pipeline_unmask(kmws_pipeline* p, uint8_t* host_base, uint64_t span, const kmws_desc* descs,
                                 uint32_t n);

/* ---- pinned host memory for the loop rings ---- */

/* Page-locked host memory for the receive / send rings (kmws_rx_batch_attach_ring,
 * kmws_tx_batch_attach_ring): hipHostMalloc'ed, visible to `device`, so a
 * caller like kuma needs no HIP headers of its own.  NULL on failure. */
void* kmws_host_alloc(size_t bytes, int device);
void  kmws_host_free(void* p);

#ifdef __cplusplus
}
#endif
#endif /* KMWS_GPU_H */
