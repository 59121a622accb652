/*
 * kmws_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of kuma's RFC 6455 frame codec (src/ws in Jamol/kuma), used
 * exclusively as the parity checker by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Nothing in kuma_amd/ links, loads or calls
 * this file; the product path is the HIP library (include/kmws_gpu.h).
 *
 * Every function cites the reference lines it restates (paths relative to the
 * reference checkout).  No reference source is copied: the byte semantics are
 * restated in plain C, including the reference's quirks.
 *
 * PARITY UNPINNED.  The reference's WSHandler.cpp cannot be compiled in this
 * image without writing stand-ins for the absent libkev headers
 * (third_party/libkev is an empty submodule), which this build does not do,
 * and the reference's own tests hold no WebSocket vectors (unittest/ covers
 * KMBuffer and Base64 only).  So no reference-held or reference-run fixture
 * checks this restatement.  What checks it (tests/golden/reference_vectors.json):
 * the RFC 6455 sec.5.7 known-answer frames -- independent of kuma, they pin the
 * protocol-defined parts (masking, the three length classes, fragmentation) --
 * and values transcribed from SURVEY.md sec.8 (a-2, a-4, a-5 tables, from a
 * survey-session build of WSHandler.cpp that needed stand-in headers: a record,
 * not a pin).  See DESIGN.md sec.2 "Oracle".
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define ORC_MAX_HEADER 14
#define ORC_MAX_FRAME_DATA_LENGTH (10u * 1024u * 1024u) /* WSHandler.cpp:110 */

/* WSError, wsdefs.h:56-67 */
enum { E_NOERR = 0, E_NEED_MORE = 1, E_HANDSHAKE = 2, E_INVALID_PARAM = 3,
       E_INVALID_STATE = 4, E_INVALID_FRAME = 5, E_INVALID_LENGTH = 6,
       E_PROTOCOL = 7, E_CLOSED = 8, E_DESTROYED = 9 };

/* WSHandler::DecodeState, WSHandler.h:57-65 */
enum { S_HDR1, S_HDR2, S_HDREX, S_MASKEY, S_DATA, S_CLOSED, S_IN_ERROR };

/* FrameHeader, wsdefs.h:74-88, flattened (bitfields -> bytes). */
typedef struct orc_hdr {
    uint8_t fin, rsv1, rsv2, rsv3, opcode, mask, plen, _pad;
    uint64_t xpl64;          /* union xpl{xpl16, xpl64}: xpl16 is its low 16 bits */
    uint8_t maskey[4];
    uint32_t length;
} orc_hdr;

/* frame callback: return nonzero to emulate "callback destroyed the handler"
 * (DESTROY_DETECTOR_CHECK, WSHandler.cpp:284-287). */
typedef int (*orc_frame_cb)(const orc_hdr* hdr, const uint8_t* payload, size_t len, void* user);

typedef struct orc_decoder {
    int mode;                /* 0 = CLIENT, 1 = SERVER (WSMode, wsdefs.h:69-72) */
    int state;
    orc_hdr hdr;
    uint8_t pos;             /* DecodeContext::pos is uint8_t (WSHandler.h:76) */
    uint8_t* buf;            /* DecodeContext::buf (std::vector<uint8_t>) */
    size_t buf_len, buf_cap;
} orc_decoder;

/* ---- a-1 / a-2: payload mask (WSHandler.cpp:303-310, chain form :312-322) ----
 * data[i] ^= key[(phase + i) % 4].  phase != 0 continues a KMBuffer chain whose
 * earlier segments held `phase` bytes.  Deliberately the reference's scalar
 * byte loop (no restrict, no vector types): it doubles as the timing twin. */
void orc_mask(const uint8_t key[4], uint8_t* data, size_t len, size_t phase)
{
    if (data == NULL || len == 0) return;                   /* :305 */
    for (size_t i = 0; i < len; ++i)
        data[i] = data[i] ^ key[(phase + i) % 4];
}

/* ---- a-4: header pack (WSHandler.cpp:46-106) ----
 * The length class is chosen from hdr->length (uint32) only; plen/xpl are
 * ignored.  127-class writes four zero bytes then the 32-bit BE length. */
int orc_encode_header(const orc_hdr* h, uint8_t out[ORC_MAX_HEADER])
{
    uint8_t b0 = (uint8_t)((h->fin ? 0x80 : 0) | (h->rsv1 ? 0x40 : 0) |
                           (h->rsv2 ? 0x20 : 0) | (h->rsv3 ? 0x10 : 0) |
                           (h->opcode & 0x0F));
    uint8_t b1 = h->mask ? 0x80 : 0;
    int n = 2;
    out[0] = b0;
    if (h->length <= 125) {                                  /* :68-71 */
        out[1] = (uint8_t)(b1 | h->length);
    } else if (h->length <= 0xFFFF) {                        /* :72-76, :85-89 */
        out[1] = b1 | 126;
        out[2] = (uint8_t)(h->length >> 8);
        out[3] = (uint8_t)h->length;
        n = 4;
    } else {                                                 /* :77-81, :90-100 */
        out[1] = b1 | 127;
        out[2] = out[3] = out[4] = out[5] = 0;
        out[6] = (uint8_t)(h->length >> 24);
        out[7] = (uint8_t)(h->length >> 16);
        out[8] = (uint8_t)(h->length >> 8);
        out[9] = (uint8_t)h->length;
        n = 10;
    }
    if (h->mask) {                                           /* :101-104 */
        memcpy(out + n, h->maskey, 4);
        n += 4;
    }
    return n;
}

/* ---- a-5: streaming decoder (WSHandler.cpp:108-280) ---- */
orc_decoder* orc_decoder_create(int mode)
{
    orc_decoder* d = (orc_decoder*)calloc(1, sizeof(orc_decoder));
    if (d) { d->mode = mode; d->state = S_HDR1; }
    return d;
}

void orc_decoder_destroy(orc_decoder* d)
{
    if (d) { free(d->buf); free(d); }
}

/* DecodeContext::reset, WSHandler.h:66-72 (capacity kept) */
void orc_decoder_reset(orc_decoder* d)
{
    memset(&d->hdr, 0, sizeof(d->hdr));
    d->state = S_HDR1;
    d->buf_len = 0;
    d->pos = 0;
}

void orc_decoder_set_mode(orc_decoder* d, int mode) { d->mode = mode; }

static int buf_append(orc_decoder* d, const uint8_t* p, size_t n)
{
    if (d->buf_len + n > d->buf_cap) {
        size_t cap = d->buf_cap ? d->buf_cap : 64;
        while (cap < d->buf_len + n) cap *= 2;
        uint8_t* nb = (uint8_t*)realloc(d->buf, cap);
        if (!nb) return -1;
        d->buf = nb;
        d->buf_cap = cap;
    }
    if (n) memcpy(d->buf + d->buf_len, p, n);
    d->buf_len += n;
    return 0;
}

static int is_control(uint8_t op) { return op >= 8; }      /* WSHandler.h:52-54 */

/* 127-class extended length, byte k of 8 (WSHandler.cpp:177-180).  The
 * reference shifts a promoted 32-bit int by (7-k)*8; on x86-64 the count is
 * taken mod 32 and the int result is sign-extended into the uint64 (SURVEY
 * sec.8 a-5, reproduced there with g++ 11.4 and clang 22 at -O0..-O3). */
static uint64_t xpl64_byte(uint8_t b, unsigned k)
{
    unsigned sh = ((7u - k) * 8u) & 31u;
    return (uint64_t)(int64_t)(int32_t)((uint32_t)b << sh);
}

int orc_decoder_feed(orc_decoder* d, uint8_t* data, size_t len, orc_frame_cb cb, void* user)
{
    size_t pos = 0;
    while (pos < len) {                                      /* :114 */
        switch (d->state) {
        case S_HDR1: {                                       /* :118-135 */
            uint8_t b = data[pos++];
            d->hdr.fin = b >> 7;
            d->hdr.opcode = b & 0x0F;
            d->hdr.rsv1 = (b >> 6) & 1;
            d->hdr.rsv2 = (b >> 5) & 1;
            d->hdr.rsv3 = (b >> 4) & 1;
            if (!d->hdr.fin && is_control(d->hdr.opcode)) {
                d->state = S_IN_ERROR;
                return E_PROTOCOL;
            }
            d->state = S_HDR2;
        } /* fallthrough */
        case S_HDR2: {                                       /* :136-156 */
            if (pos < len) {
                uint8_t b = data[pos++];
                d->hdr.mask = b >> 7;
                d->hdr.plen = b & 0x7F;
                d->hdr.xpl64 = 0;
                d->pos = 0;
                d->buf_len = 0;
                if (is_control(d->hdr.opcode) && d->hdr.plen > 125) {
                    d->state = S_IN_ERROR;
                    return E_PROTOCOL;
                }
                d->state = S_HDREX;
            } else {
                return E_NEED_MORE;
            }
        } /* fallthrough */
        case S_HDREX: {                                      /* :157-204 */
            if (d->hdr.plen == 126) {
                for (; pos < len && d->pos < 2; ++pos, ++d->pos) {
                    uint16_t x16 = (uint16_t)d->hdr.xpl64;
                    x16 = (uint16_t)(x16 | (data[pos] << ((2 - d->pos - 1) << 3)));
                    d->hdr.xpl64 = (d->hdr.xpl64 & ~(uint64_t)0xFFFF) | x16;
                }
                if (d->pos >= 2) {
                    d->pos = 0;
                    uint16_t x16 = (uint16_t)d->hdr.xpl64;
                    if (x16 < 126) { d->state = S_IN_ERROR; return E_INVALID_LENGTH; }
                    d->hdr.length = x16;
                    d->state = S_MASKEY;
                } else {
                    return E_NEED_MORE;
                }
            } else if (d->hdr.plen == 127) {
                for (; pos < len && d->pos < 8; ++pos, ++d->pos)
                    d->hdr.xpl64 |= xpl64_byte(data[pos], d->pos);
                if (d->pos >= 8) {
                    d->pos = 0;
                    if ((d->hdr.xpl64 >> 63) != 0) { d->state = S_IN_ERROR; return E_INVALID_LENGTH; }
                    d->hdr.length = (uint32_t)d->hdr.xpl64;
                    if (d->hdr.length > ORC_MAX_FRAME_DATA_LENGTH) {
                        d->state = S_IN_ERROR;
                        return E_INVALID_LENGTH;
                    }
                    d->state = S_MASKEY;
                } else {
                    return E_NEED_MORE;
                }
            } else {
                d->hdr.length = d->hdr.plen;
                d->state = S_MASKEY;
            }
        } /* fallthrough */
        case S_MASKEY: {                                     /* :205-234 */
            if (d->hdr.mask) {
                if (d->mode == 0) { d->state = S_IN_ERROR; return E_PROTOCOL; }
                size_t copy_len = 4u - d->pos;
                if (copy_len > len - pos) copy_len = len - pos;
                memcpy(d->hdr.maskey + d->pos, data + pos, copy_len);
                pos += copy_len;
                d->pos = (uint8_t)(d->pos + copy_len);
                if (d->pos < 4) return E_NEED_MORE;
                d->pos = 0;
            } else if (d->mode == 1 && d->hdr.length > 0) {
                d->state = S_IN_ERROR;
                return E_PROTOCOL;
            }
            d->buf_len = 0;
            d->state = S_DATA;
        } /* fallthrough */
        case S_DATA: {                                       /* :235-272 */
            if (len - pos + d->buf_len < d->hdr.length) {
                if (buf_append(d, data + pos, len - pos)) return E_INVALID_STATE;
                return E_NEED_MORE;
            }
            uint8_t* nd;
            uint32_t nl = d->hdr.length;
            if (d->buf_len == 0) {
                nd = data + pos;
                pos += nl;
            } else {
                size_t read_len = d->hdr.length - d->buf_len;
                if (buf_append(d, data + pos, read_len)) return E_INVALID_STATE;
                nd = d->buf;
                pos += read_len;
            }
            if (d->hdr.mask) orc_mask(d->hdr.maskey, nd, nl, 0);   /* :260, :291-295 */
            if (cb && cb(&d->hdr, nd, nl, user)) return E_DESTROYED; /* :261, :282-289 */
            if (d->hdr.opcode == 8) {                        /* :265-268 */
                d->state = S_CLOSED;
                return E_CLOSED;
            }
            orc_decoder_reset(d);                            /* :270 */
            break;
        }
        default:
            return E_INVALID_FRAME;                          /* :273-276 */
        }
    }
    return d->state == S_HDR1 ? E_NOERR : E_NEED_MORE;       /* :279 */
}

int orc_decoder_state(const orc_decoder* d) { return d->state; }

/* ---- batch helpers used by the GPU parity tests and the CPU baseline ---- */

/* Mirror of kmws_desc (include/kmws_gpu.h). */
typedef struct orc_desc { uint64_t off; uint32_t len; uint32_t key; } orc_desc;

/* Unmask every frame of a descriptor batch in place, one frame at a time, with
 * the reference's byte loop (a-1).  key is the little-endian u32 of the four
 * wire key bytes, i.e. the bytes of hdr.maskey in memory order. */
void orc_unmask_batch(uint8_t* base, const orc_desc* descs, size_t n)
{
    for (size_t i = 0; i < n; ++i) {
        uint8_t k[4];
        memcpy(k, &descs[i].key, 4);
        orc_mask(k, base + descs[i].off, descs[i].len, 0);
    }
}

typedef struct mt_arg { uint8_t* base; const orc_desc* d; size_t n; } mt_arg;

static void* mt_body(void* p)
{
    mt_arg* a = (mt_arg*)p;
    orc_unmask_batch(a->base, a->d, a->n);
    return NULL;
}

/* Same work split over nthreads pthreads, frames partitioned contiguously
 * (one independent handler per thread, as SURVEY sec.8 d measures kuma). */
int orc_unmask_batch_mt(uint8_t* base, const orc_desc* descs, size_t n, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    mt_arg args[256];
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    int started = 0;
    for (int t = 0; t < nthreads; ++t) {
        size_t lo = (size_t)t * per, hi = lo + per;
        if (lo >= n) break;
        if (hi > n) hi = n;
        args[t].base = base; args[t].d = descs + lo; args[t].n = hi - lo;
        if (pthread_create(&th[t], NULL, mt_body, &args[t]) != 0) return -1;
        ++started;
    }
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    return started;
}

/* Out-of-place encode of a batch (a-10 composition: header pack then masked
 * payload, WebSocketImpl.cpp:381-404): frame i takes payload bytes
 * src[src_off[i] .. +len) and writes header||payload at dst + wire_off[i],
 * where wire_off is the running sum of (hdr_len + len).  flags bit layout as
 * kmws_frame_flags in include/kmws_gpu.h: bit7 fin, bit6 rsv1, bit5 rsv2,
 * bit4 rsv3, bits0-3 opcode, bit8 mask.  Returns total wire bytes. */
uint64_t orc_encode_batch(const uint8_t* src, const uint64_t* src_off, const uint32_t* lens,
                          const uint32_t* flags, const uint32_t* keys, size_t n,
                          uint8_t* dst, uint64_t* wire_off)
{
    uint64_t w = 0;
    for (size_t i = 0; i < n; ++i) {
        orc_hdr h;
        memset(&h, 0, sizeof(h));
        h.fin = (flags[i] >> 7) & 1; h.rsv1 = (flags[i] >> 6) & 1;
        h.rsv2 = (flags[i] >> 5) & 1; h.rsv3 = (flags[i] >> 4) & 1;
        h.opcode = flags[i] & 0x0F; h.mask = (flags[i] >> 8) & 1;
        memcpy(h.maskey, &keys[i], 4);
        h.length = lens[i];
        if (wire_off) wire_off[i] = w;
        uint8_t hb[ORC_MAX_HEADER];
        int hl = orc_encode_header(&h, hb);
        if (dst) {
            memcpy(dst + w, hb, (size_t)hl);
            memcpy(dst + w + hl, src + src_off[i], lens[i]);
            if (h.mask) orc_mask(h.maskey, dst + w + hl, lens[i], 0);
        }
        w += (uint64_t)hl + lens[i];
    }
    return w;
}
