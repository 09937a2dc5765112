#ifndef WS_COMMON_H
#define WS_COMMON_H

/*
 * netc WebSocket framing API — declarations and struct layouts identical to the
 * reference's include/ws/common.h (Altanis/netc @ 2024-08-07), so code written
 * against netc compiles and links unchanged against this library:
 *   opcodes            include/ws/common.h:34-39
 *   parse errors       include/ws/common.h:42-50
 *   parse states       include/ws/common.h:53-67
 *   struct ws_header   include/ws/common.h:70-82   (1 byte of bitfields)
 *   struct ws_frame    include/ws/common.h:85-97
 *   struct ws_message  include/ws/common.h:100-108
 *   struct ws_frame_parsing_state  include/ws/common.h:111-127  (embedded by
 *                      value in struct web_client and memset by callers: ABI)
 *   functions          include/ws/common.h:130-137
 * The masking inner loops now go through include/ws/mask.h.
 *
 * Wire format, RFC 6455 §5.2:
 *   byte 0  FIN | RSV1 | RSV2 | RSV3 | opcode(4)
 *   byte 1  MASK | payload len(7)      (126 → 16-bit, 127 → 64-bit length follows, big endian)
 *   [4 byte masking key if MASK]       payload
 */

#include "../utils/vector.h"

#include <stdint.h>
#include <stddef.h>
#include <stdbool.h>

#define WEBSOCKET_HANDSHAKE_GUID "258EAFA5-E914-47DA-95CA-C5AB0DC85B11"
#define WEBSOCKET_VERSION "13"

#define WS_OPCODE_CONTINUE 0x0
#define WS_OPCODE_TEXT     0x1
#define WS_OPCODE_BINARY   0x2
#define WS_OPCODE_CLOSE    0x8
#define WS_OPCODE_PING     0x9
#define WS_OPCODE_PONG     0xA

struct web_client;

/** Errors returned by ws_parse_frame. */
enum ws_frame_parsing_errors
{
    /** The `recv` syscall failed. */
    WS_FRAME_PARSE_ERROR_RECV = -1,
    /** The payload length for the frame is invalid. */
    WS_FRAME_PARSE_ERROR_INVALID_FRAME_LENGTH = -2,
    /** The payload length is too big. */
    WS_FRAME_PARSE_ERROR_PAYLOAD_TOO_BIG = -3
};

/** Where the incremental parser is inside the current frame. */
enum ws_frame_parsing_states
{
    WS_FRAME_NIL = -1,
    WS_FRAME_PARSING_STATE_FIRST_BYTE,
    WS_FRAME_PARSING_STATE_SECOND_BYTE,
    WS_FRAME_PARSING_STATE_PAYLOAD_LENGTH,
    WS_FRAME_PARSING_STATE_MASKING_KEY,
    WS_FRAME_PARSING_STATE_PAYLOAD_DATA
};

/** First byte of a frame. */
struct ws_header
{
    uint8_t fin:     1;
    uint8_t rsv1:    1;
    uint8_t rsv2:    1;
    uint8_t rsv3:    1;
    uint8_t opcode:  4;
};

/** One frame being parsed. */
struct ws_frame
{
    struct ws_header header;
    /** MASK bit of the second byte. */
    bool mask;
    /** The 4 key bytes in wire order. */
    uint8_t masking_key[4];
    /** The 7-bit length field of the second byte (126/127 = extended). */
    uint64_t payload_length;
};

/** A complete (reassembled) message. */
struct ws_message
{
    uint8_t opcode;
    /** Payload; owned by the caller once ws_parse_frame returned 0. */
    uint8_t *buffer;
    size_t payload_length;
};

/** Per-connection parser state; zero-initialise (or memset) to start. */
struct ws_frame_parsing_state
{
    enum ws_frame_parsing_states parsing_state;

    struct ws_frame frame;
    struct ws_message message;

    /** Decoded payload length of the current frame. */
    uint64_t real_payload_length;
    /** Reassembly buffer for the message (all frames' payloads back to back). */
    struct vector payload_data;
    /** Payload bytes of the current frame received so far (the masking phase). */
    size_t received_length;
};

/** Fills a masking key (deterministic per-thread sequence, as the reference: src/ws/common.c:19-27). */
void ws_build_masking_key(uint8_t masking_key[4]);
/** Describes a message; borrows payload_data. */
void ws_build_message(struct ws_message *message, uint8_t opcode, uint64_t payload_length, uint8_t *payload_data);

/** Sends a message split into num_frames frames, masked when masking_key != NULL. Returns 1, else the failing send() result. */
int ws_send_message(struct web_client *client, struct ws_message *message, uint8_t masking_key[4], size_t num_frames);
/** Parses incoming frames. 0 = message complete in state->message, 1 = need more data, < 0 = enum ws_frame_parsing_errors. */
int ws_parse_frame(struct web_client *client, struct ws_frame_parsing_state *current_state, size_t MAX_PAYLOAD_LENGTH);

#endif // WS_COMMON_H
