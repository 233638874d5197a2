"""AMQP 0-9-1 protocol layer: constants, method table, golden codec."""
from . import constants
from .codec import (CodecError, Command, CommandAssembler, Frame, FrameParser, Method, Reader, Typed,
                    Writer, decode_content_header, decode_method, decode_properties, decode_table,
                    encode_content_header, encode_frame, encode_method_frame, encode_properties,
                    encode_table, render_command)
from .methods import BASIC_PROPERTIES, BY_ID, BY_NAME, METHODS
