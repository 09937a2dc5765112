/*
 * WebSocket framing for netc: frame encoder (ws_send_message) and incremental
 * frame parser (ws_parse_frame), rebuilt around the masking C-ABI of
 * include/ws/mask.h.  Same API, return codes, buffer ownership and parser
 * state layout as the reference (include/ws/common.h:129-137,
 * src/ws/common.c:19-348); the per-byte masking loops of the reference
 * (src/ws/common.c:104-107 and :317-323) are replaced by netc_ws_mask, which is
 * RFC 6455 §5.3 exactly: out[i] = in[i] ^ key[(phase + i) & 3].
 *
 * Intentional differences from the reference (see DESIGN.md "Reference
 * defects"): every frame of a multi-frame masked send carries its own masked
 * slice (B2); masked binary payloads of any length (B1) and TEXT payloads with
 * embedded NULs (B3) are sent from payload_length, not strlen / the header
 * byte; frames are assembled on the heap, not a stack VLA (B4); short writes
 * are completed without waiting for the peer: what a non-blocking socket does not
 * take is kept in the connection's send backlog (include/ws/route.h) (B5); a masked empty payload still carries its key (RFC 6455
 * §5.2); a recv() error no longer corrupts the buffer bookkeeping (B6); split
 * masking keys / extended lengths are resumed by byte count, not by a zero-byte
 * heuristic (B7, B8).
 */
#include "../../../include/ws/common.h"
#include "../../../include/ws/mask.h"
#include "../../../include/ws/route.h"
#include "../../../include/tcp/server.h"
#include "../../../include/utils/error.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/uio.h>

/*
 * struct web_client (reference include/web/client.h:12-100) begins with
 * `struct tcp_client *tcp_client`; the WebSocket path reads nothing else from
 * it (src/ws/common.c:38,136), so only that leading member is named here.
 */
struct web_client_head
{
    struct tcp_client *tcp_client;
};

static socket_t client_socket(struct web_client *client)
{
    return ((struct web_client_head *)client)->tcp_client->sockfd;
}

/* ------------------------------------------------------------------ keys -- */

static __thread int key_seed = 0;

void ws_build_masking_key(uint8_t masking_key[4])
{
    /* the reference's deterministic per-thread sequence (src/ws/common.c:19-27):
       byte j of call c on a fresh thread is (uint8_t)(97 * (4c + j)) */
    for (int j = 0; j < 4; ++j) masking_key[j] = (uint8_t)(key_seed++ * 97);
}

void ws_build_message(struct ws_message *message, uint8_t opcode, uint64_t payload_length, uint8_t *payload_data)
{
    message->opcode = opcode;
    message->payload_length = payload_length;
    message->buffer = payload_data;
}

/* ------------------------------------------------------------------ send -- */

/* header of one frame into out (<= 14 bytes); returns its length */
static size_t encode_header(uint8_t *out, int fin, uint8_t opcode, const uint8_t *key, uint64_t len)
{
    size_t h = 0;
    out[h++] = (uint8_t)((fin ? 0x80 : 0x00) | (opcode & 0x0F));
    const uint8_t mbit = key ? 0x80 : 0x00;
    if (len <= 125)
        out[h++] = (uint8_t)(mbit | len);
    else if (len <= 0xFFFF)
    {
        out[h++] = (uint8_t)(mbit | 126);
        out[h++] = (uint8_t)(len >> 8);
        out[h++] = (uint8_t)len;
    }
    else
    {
        out[h++] = (uint8_t)(mbit | 127);
        for (int i = 7; i >= 0; --i) out[h++] = (uint8_t)(len >> (8 * i));
    }
    if (key)
    {
        memcpy(out + h, key, 4);
        h += 4;
    }
    return h;
}

int ws_send_message(struct web_client *client, struct ws_message *message, uint8_t masking_key[4], size_t num_frames)
{
    const socket_t fd = client_socket(client);

    /* a connection with a send route attached (include/ws/route.h: e.g. the GPU egress ring,
       netc_ws_gpu_attach_send) is served by it, with this function's contract */
    void *route_ctx = NULL;
    const netc_ws_send_route_fn route = netc_ws_send_route_get((int)fd, &route_ctx);
    if (route) return route(route_ctx, (int)fd, message, masking_key, num_frames);

    if (num_frames == 0) num_frames = 1;

    /* frame sizes as the reference (src/ws/common.c:42-49): equal split, remainder on the last frame */
    const uint64_t total = message->payload_length;
    const uint64_t split = total / num_frames, rem = total % num_frames;
    const uint8_t *payload = message->buffer;
    uint64_t passed = 0;

    for (size_t i = 0; i < num_frames; ++i)
    {
        const int last = i + 1 == num_frames;
        const uint64_t flen = split + (last ? rem : 0);
        uint8_t hdr[14];
        const size_t hlen = encode_header(hdr, last, i == 0 ? message->opcode : WS_OPCODE_CONTINUE, masking_key, flen);
        int r;
        if (masking_key != NULL && flen != 0)
        {
            /* header + masked copy of this frame's own slice, assembled in one pass */
            uint8_t *frame = malloc(hlen + flen);
            if (frame == NULL)
            {
                errno = ENOMEM;
                (void)netc_error(BADSEND);
                return -1;
            }
            memcpy(frame, hdr, hlen);
            netc_ws_mask(frame + hlen, payload + passed, (size_t)flen, masking_key, 0);
            struct iovec iov[1] = {{frame, hlen + flen}};
            r = netc_ws_send_nb((int)fd, iov, 1, 0);
            free(frame);
        }
        else
        {
            struct iovec iov[2] = {{hdr, hlen}, {(void *)(payload + passed), (size_t)flen}};
            r = netc_ws_send_nb((int)fd, iov, flen ? 2 : 1, 0);
        }
        if (r <= 0) return r;
        passed += flen;
    }
    return 1;
}

/* ----------------------------------------------------------------- parse -- */

/* one recv(); 0 with *got > 0 on data, 1 when it would block, < 0 on error / EOF */
static int recv_some(socket_t fd, void *buf, size_t n, size_t *got)
{
    for (;;)
    {
        const ssize_t r = recv(fd, buf, n, 0);
        if (r > 0)
        {
            *got = (size_t)r;
            return 0;
        }
        if (r == 0) return WS_FRAME_PARSE_ERROR_RECV; /* peer closed */
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) return 1;
        (void)netc_error(BADRECV);
        return WS_FRAME_PARSE_ERROR_RECV;
    }
}

int ws_parse_frame(struct web_client *client, struct ws_frame_parsing_state *st, size_t MAX_PAYLOAD_LENGTH)
{
    const socket_t fd = client_socket(client);
    size_t got = 0;
    int r;

    /* a connection with a receive route attached (include/ws/route.h: e.g. the GPU ingest ring,
       netc_ws_gpu_attach) is served by it, with this function's contract */
    void *route_ctx = NULL;
    const netc_ws_route_fn route = netc_ws_route_get((int)fd, &route_ctx);
    /* the connection is readable: a send backlog it holds goes out first, without waiting */
    if (netc_ws_send_pending((int)fd) > 0) (void)netc_ws_send_flush((int)fd);
    if (route) return route(route_ctx, (int)fd, st, MAX_PAYLOAD_LENGTH);

    for (;;)
    {
        switch (st->parsing_state)
        {
        case WS_FRAME_NIL:
            st->parsing_state = WS_FRAME_PARSING_STATE_FIRST_BYTE;
            break;

        case WS_FRAME_PARSING_STATE_FIRST_BYTE:
        {
            uint8_t b;
            if ((r = recv_some(fd, &b, 1, &got)) != 0) return r;
            st->frame.header.fin = (b >> 7) & 1;
            st->frame.header.rsv1 = (b >> 6) & 1;
            st->frame.header.rsv2 = (b >> 5) & 1;
            st->frame.header.rsv3 = (b >> 4) & 1;
            st->frame.header.opcode = b & 0x0F;
            if (st->frame.header.opcode != WS_OPCODE_CONTINUE) st->message.opcode = st->frame.header.opcode;
            st->parsing_state = WS_FRAME_PARSING_STATE_SECOND_BYTE;
            break;
        }

        case WS_FRAME_PARSING_STATE_SECOND_BYTE:
        {
            uint8_t b;
            if ((r = recv_some(fd, &b, 1, &got)) != 0) return r;
            st->frame.mask = (b >> 7) & 1;
            st->frame.payload_length = b & 0x7F;
            st->real_payload_length = 0;
            st->received_length = 0; /* counts extended-length bytes next */
            st->parsing_state = WS_FRAME_PARSING_STATE_PAYLOAD_LENGTH;
            break;
        }

        case WS_FRAME_PARSING_STATE_PAYLOAD_LENGTH:
        {
            if (st->frame.payload_length <= 125)
                st->real_payload_length = st->frame.payload_length;
            else
            {
                /* 16- or 64-bit big-endian length, resumable across recv boundaries */
                const size_t need = st->frame.payload_length == 126 ? 2 : 8;
                while (st->received_length < need)
                {
                    uint8_t buf[8];
                    if ((r = recv_some(fd, buf, need - st->received_length, &got)) != 0) return r;
                    for (size_t i = 0; i < got; ++i) st->real_payload_length = (st->real_payload_length << 8) | buf[i];
                    st->received_length += got;
                }
                if (need == 8 && (st->real_payload_length >> 63) != 0) return WS_FRAME_PARSE_ERROR_INVALID_FRAME_LENGTH;
            }
            st->received_length = 0;

            if (st->real_payload_length > MAX_PAYLOAD_LENGTH ||
                st->payload_data.size > MAX_PAYLOAD_LENGTH - st->real_payload_length)
                return WS_FRAME_PARSE_ERROR_PAYLOAD_TOO_BIG;
            if (st->payload_data.elements == NULL)
                vector_init(&st->payload_data, st->real_payload_length + (st->message.opcode == WS_OPCODE_TEXT ? 1 : 0), sizeof(uint8_t));
            st->message.payload_length = st->real_payload_length;
            if (st->frame.mask) memset(st->frame.masking_key, 0, sizeof(st->frame.masking_key));
            st->parsing_state = st->frame.mask ? WS_FRAME_PARSING_STATE_MASKING_KEY : WS_FRAME_PARSING_STATE_PAYLOAD_DATA;
            break;
        }

        case WS_FRAME_PARSING_STATE_MASKING_KEY:
        {
            while (st->received_length < 4)
            {
                if ((r = recv_some(fd, st->frame.masking_key + st->received_length, 4 - st->received_length, &got)) != 0) return r;
                st->received_length += got;
            }
            st->received_length = 0; /* payload phase starts at 0 */
            st->parsing_state = WS_FRAME_PARSING_STATE_PAYLOAD_DATA;
            break;
        }

        case WS_FRAME_PARSING_STATE_PAYLOAD_DATA:
        {
            if (st->real_payload_length == 0) goto frame_done;
            const uint64_t remaining = st->real_payload_length - st->received_length;
            if (st->payload_data.capacity < st->payload_data.size + remaining)
            {
                vector_resize(&st->payload_data, st->payload_data.size + remaining);
                if (st->payload_data.capacity < st->payload_data.size + remaining) return WS_FRAME_PARSE_ERROR_PAYLOAD_TOO_BIG;
            }
            uint8_t *dst = (uint8_t *)st->payload_data.elements + st->payload_data.size;
            if ((r = recv_some(fd, dst, (size_t)remaining, &got)) != 0) return r;
            /* unmask in place; the phase is this frame's bytes already received (src/ws/common.c:321) */
            if (st->frame.mask) netc_ws_mask(dst, dst, got, st->frame.masking_key, st->received_length);
            st->payload_data.size += got;
            st->received_length += got;
            if (got < remaining) return 1;
            goto frame_done;
        }

        default:
            return WS_FRAME_PARSE_ERROR_INVALID_FRAME_LENGTH;
        }
    }

frame_done:
{
    const int fin = st->frame.header.fin;
    st->parsing_state = WS_FRAME_NIL;
    st->real_payload_length = 0;
    st->received_length = 0;
    memset(&st->frame, 0, sizeof(st->frame));
    if (!fin) return 1;
    if (st->message.opcode == WS_OPCODE_TEXT) vector_push(&st->payload_data, &(char){'\0'});
    st->message.payload_length = st->payload_data.size;
    st->message.buffer = st->payload_data.elements;
    return 0;
}
}
