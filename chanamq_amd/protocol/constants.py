"""AMQP 0-9-1 wire constants.

Parity notes (reference = ChanaMQ, /root/reference):
  * frame types / end marker / heartbeat bytes: chana-mq-base/.../model/Frame.scala:40-77
  * protocol header 'AMQP' 0 0 9 1:              chana-mq-base/.../model/AMQProtocol.scala:11-39
  * reply codes:                                  chana-mq-base/.../model/ErrorCodes.scala:5-112
  * exchange types:                               chana-mq-base/.../model/AMQP.scala:24-46
"""

PROTOCOL_HEADER = b"AMQP\x00\x00\x09\x01"

FRAME_METHOD = 1
FRAME_HEADER = 2
FRAME_BODY = 3
FRAME_HEARTBEAT = 8
FRAME_END = 0xCE
FRAME_NON_BODY_SIZE = 8  # type(1) + channel(2) + size(4) + end(1)
HEARTBEAT_FRAME = bytes([8, 0, 0, 0, 0, 0, 0, 0xCE])

# class ids
CONNECTION = 10
CHANNEL = 20
ACCESS = 30
EXCHANGE = 40
QUEUE = 50
BASIC = 60
CONFIRM = 85
TX = 90

# reply codes (ErrorCodes.scala)
REPLY_SUCCESS = 200
CONTENT_TOO_LARGE = 311
NO_ROUTE = 312
NO_CONSUMERS = 313
CONNECTION_FORCED = 320
INVALID_PATH = 402
ACCESS_REFUSED = 403
NOT_FOUND = 404
RESOURCE_LOCKED = 405
PRECONDITION_FAILED = 406
FRAME_ERROR = 501
SYNTAX_ERROR = 502
COMMAND_INVALID = 503
CHANNEL_ERROR = 504
UNEXPECTED_FRAME = 505
RESOURCE_ERROR = 506
NOT_ALLOWED = 530
NOT_IMPLEMENTED = 540
INTERNAL_ERROR = 541

REPLY_TEXT = {
    200: "OK",
    311: "CONTENT_TOO_LARGE",
    312: "The exchange cannot route the result of a Publish",  # ErrorCodes.scala:23-27 (NO_ROUTE text)
    313: "The exchange cannot deliver to a consumer when the immediate flag is set",
    320: "CONNECTION_FORCED",
    402: "INVALID_PATH",
    403: "ACCESS_REFUSED",
    404: "NOT_FOUND",
    405: "RESOURCE_LOCKED",
    406: "PRECONDITION_FAILED",
    501: "FRAME_ERROR",
    502: "SYNTAX_ERROR",
    503: "COMMAND_INVALID",
    504: "CHANNEL_ERROR",
    505: "UNEXPECTED_FRAME",
    506: "RESOURCE_ERROR",
    530: "NOT_ALLOWED",
    540: "NOT_IMPLEMENTED",
    541: "INTERNAL_ERROR",
}

EXCHANGE_TYPES = ("direct", "fanout", "topic", "headers")
EX_DIRECT, EX_FANOUT, EX_TOPIC, EX_HEADERS = 0, 1, 2, 3
EXCHANGE_TYPE_ID = {"direct": EX_DIRECT, "fanout": EX_FANOUT, "topic": EX_TOPIC, "headers": EX_HEADERS}

DEFAULT_PORT = 5672
DEFAULT_TLS_PORT = 5671

# server identity sent in Connection.Start (FrameStage.scala:200-215)
SERVER_PROPERTIES = {"product": "chana.mq", "version": "0.1.0", "chana.mq.build": "1"}
SERVER_MECHANISMS = "PLAIN"
SERVER_LOCALES = "en_US"
