// Message bodies of the GPU write-behind path (BASELINE config 4) in striped, append-only
// segment files next to the store's WAL.
//
// The WAL keeps the rows (store.hpp); a persistent message's bytes -- the device's packed
// persist record (step_abi.h PersistHdr + exchange | routing key | properties | body) --
// are written once, straight from the step's record buffer, by one of `stripes` writer
// threads with pwritev, and the WAL row carries only (segment, offset, length).  A group
// commit starts the body writes, appends and fsyncs the WAL meanwhile, then waits for the
// stripes' own fdatasync: confirms leave after both.  Each record is framed with a CRC-32C
// so recovery refuses a torn body (such a message was never confirmed).
//
// The reference writes each message row to Cassandra (CassandraOpService.scala:395-417
// insertMessage), which spreads the writes over its memtables / commitlog; here the
// spreading is the stripes, and a segment file is unlinked once no live row refers to it.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace cmq {

uint32_t crc32c(const char* p, size_t n);

class BodyLog {
 public:
  struct Loc { uint32_t seg = 0, len = 0; uint64_t off = 0; };   // off: the record's frame
  struct Stats {
    uint64_t written = 0, records = 0, live_bytes = 0, live_records = 0, disk_bytes = 0, segments = 0,
             reclaimed = 0, bad_reads = 0;
    double write_s = 0, sync_s = 0;
  };
  static constexpr uint32_t FRAME = 16;   // u32 magic | u32 len | u32 crc | u32 0

  BodyLog(std::string dir, bool fsync);
  ~BodyLog();
  void configure(int stripes, uint64_t seg_bytes);
  // a byte budget shared with the WAL (Store::set_quota): a put() past it fails like a full
  // disk (the sticky error wait() reports), nothing of it is written
  void set_quota(std::atomic<uint64_t>* used, uint64_t limit) { q_used_ = used; q_lim_ = limit; }
  // place n records (locations returned now) and start writing them; the pointers must stay
  // valid until wait() returns
  void put(const char* const* recs, const uint32_t* lens, size_t n, Loc* out);
  bool wait(std::string* err);           // every put() so far written (and fdatasync'd)
  void ref(const Loc& l);
  void unref(const Loc& l);
  void reap();                           // unlink segments without live records
  bool read(const Loc& l, std::string* rec);
  void open_existing();                  // after the WAL replay: drop dead segments
  Stats stats();
  void close();
  const std::string& dir() const { return dir_; }

 private:
  struct Seg { uint64_t live_n = 0, live_bytes = 0, size = 0; int rfd = -1; bool current = false; };
  struct Job { int fd; uint64_t off; std::vector<const char*> recs; std::vector<uint32_t> lens; };
  struct Stripe {
    std::thread th;
    std::deque<Job> q;
    int fd = -1;
    uint32_t seg = 0;
    uint64_t off = 0;
    std::vector<int> retired;          // fds of rolled segments: closed after their last sync
  };
  void start_locked();
  void roll_locked(Stripe& s);
  void sync_dir_locked();
  void run(int k);
  std::string path(uint32_t seg) const;

  std::string dir_;
  bool fsync_;
  int dfd_ = -1;                     // the bodies directory (fsync after segment creation)
  int nstripes_ = 4;
  uint64_t seg_bytes_ = 1ull << 30;
  std::mutex mu_;                        // stripes, jobs
  std::condition_variable cv_, done_cv_;
  std::vector<Stripe> st_;
  bool started_ = false, stop_ = false;
  uint64_t pending_ = 0;
  std::string err_;
  std::atomic<uint64_t>* q_used_ = nullptr;
  uint64_t q_lim_ = 0;
  int rr_ = 0;
  uint32_t next_seg_ = 1;
  std::mutex amu_;                       // segment accounting, read fds
  std::unordered_map<uint32_t, Seg> segs_;
  std::vector<uint32_t> dead_;
  Stats stats_;
  // reaped segments are closed and unlinked by their own thread: freeing a GB-sized file's
  // pages takes 10s-100s of ms, which in the store thread held every confirm (config 4's
  // 0.3 s stalls every ~1.8 s, profiles/r5_c4/)
  void reaper();
  std::thread reap_th_;
  std::mutex rmu_;
  std::condition_variable rcv_;
  std::deque<std::pair<int, std::string>> reap_q_;
  bool reap_stop_ = false;
};

}  // namespace cmq
