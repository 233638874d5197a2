"""chanamq_amd — an MI355X-native AMQP 0-9-1 broker.

Layers:
  protocol/  golden AMQP codec (Python)            client/   AMQP test client + load generator
  models/    exchanges, queues, bindings, matchers  ops/      HIP (gfx950) data-plane kernels
  engine/    GPU data plane (hipGraph step)         parallel/ queue sharding over RCCL, HA
  broker/    C++ control plane + CPU data plane     store/    Cassandra-schema embedded store
  server/    launcher + admin REST                  utils/    config, snowflake ids, metrics
"""
__version__ = "0.1.0"
