// PerfTest-shaped native load generator (see loadgen.cpp).
#pragma once
#include <string>

namespace cmq {

struct LoadSpec {
  std::string host = "127.0.0.1";
  int port = 5672;
  std::string vhost = "/";
  int producers = 1, consumers = 1;
  int msg_size = 256;
  double seconds = 5;
  std::string exchange = "lg.direct", exchange_type = "direct", routing_key = "lg", queue = "lg.q";
  int queues = 1;
  bool auto_ack = true;
  int prefetch = 5000;
  bool persistent = false, durable = false, confirm = false;
  double rate = 0;   // msgs/s per producer, 0 = unthrottled
  int threads = 0;   // epoll worker threads (0 = min(8, connections))
  double warmup = 0; // seconds excluded from the counts
  int confirm_window = 0;    // confirm mode: max unconfirmed publishes per producer (PerfTest -c), 0 = unlimited
  int consumer_threads = 0;  // of `threads`, serving consumers (0 = half)
  int nack_every = 0;        // manual ack: every n-th ack of a consumer is Basic.Nack(multiple,
                             // requeue) instead (redelivery storm, BASELINE config 5)
  // sharded broker: the topology is declared through `port` (queues live on that rank);
  // consumers / producers may attach to other ranks (0 = `port`)
  int consumer_port = 0, producer_port = 0;
};

struct LoadResult {
  unsigned long long sent = 0, received = 0, confirmed = 0, nacked = 0;
  unsigned long long redelivered = 0;   // deliveries flagged redelivered (within received)
  unsigned long long requeued = 0;      // messages the consumers nacked back (nack_every)
  unsigned long long flow_off = 0;      // Channel.Flow(active=false) received by producers
  int threads = 0;
  double cpu_consumers_s = 0, cpu_producers_s = 0;   // thread CPU time of the load generator
  double elapsed = 0, p50_us = 0, p95_us = 0, p99_us = 0;
  std::string error;
};

LoadResult run_load(const LoadSpec& s);

}  // namespace cmq
