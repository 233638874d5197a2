"""AMQP 0-9-1 test client + load generators."""
from .amqp_client import ChannelClosed, Connection, ConnectionClosed, Delivery
