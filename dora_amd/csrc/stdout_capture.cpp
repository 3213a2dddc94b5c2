// send_stdout_as: the node library, not the daemon, owns the capture here (the daemon of this
// build does not spawn nodes).  Like the reference's spawn.rs:280-437, each batch of lines —
// one line, or for tracing output (TRACE/DEBUG/INFO/WARN/ERROR) every line up to an empty
// line — becomes `String::into_arrow()` (a Utf8 array of one element, trailing newline kept),
// is packed with required_data_size / copy_array_into_sample (dora::build_plan + host copies)
// and sent as an inline `DataMessage::Vec` sample, whatever its size, as the daemon's Logs
// event does.
#include "stdout_capture.h"

#include <unistd.h>

#include <cstring>
#include <thread>

#include "plan.h"
#include "shm.h"
#include "wire.h"

namespace dora {

class StdoutCapture {
 public:
  std::string output;
  RequestFn request;
  int saved[2] = {-1, -1};  // original fd 1 / fd 2
  int wfd[2] = {-1, -1};    // write ends now installed as fd 1 / fd 2
  std::thread readers[2];
};

namespace {

// One log batch on `output`: a Utf8 array [text] packed like any other array.
void send_batch(StdoutCapture* c, const std::string& text) {
  const int32_t offsets[2] = {0, static_cast<int32_t>(text.size())};
  const void* bufs[3] = {nullptr, offsets, text.data()};
  ArrowArray a{};
  a.length = 1;
  a.n_buffers = 3;
  a.buffers = bufs;
  ArrowSchema s{};
  s.format = "u";
  s.name = "";
  dora_plan* plan = nullptr;
  if (build_plan(&a, &s, ARROW_DEVICE_CPU, &plan) != DORA_OK) return;
  DataMsg d;
  d.kind = DATA_VEC;
  d.vec.assign(plan->size, 0);
  for (const Segment& g : plan->segs) std::memcpy(d.vec.data() + g.dst_off, g.src, g.len);
  WBuf m;
  Metadata md;
  md.timestamp_ns = now_ns();
  serialize_type_info(plan->root, md.type_info);
  delete plan;
  m.metadata(md);
  WBuf w;
  w.str(c->output);
  w.bytes(m.data(), m.size());
  w.data(d);
  (void)c->request(REQ_SEND_MESSAGE, w.take());
}

bool tracing_output(const std::string& s) {
  for (const char* k : {"TRACE", "INFO", "DEBUG", "WARN", "ERROR"})
    if (s.find(k) != std::string::npos) return true;
  return false;
}

void pump(StdoutCapture* c, int rfd, int tee) {
  std::string buf, batch;
  char tmp[4096];
  for (;;) {
    const ssize_t k = read(rfd, tmp, sizeof(tmp));
    if (k <= 0) break;
    for (ssize_t off = 0; off < k;) {  // the original descriptor still gets every byte
      const ssize_t wr = write(tee, tmp + off, size_t(k - off));
      if (wr <= 0) break;
      off += wr;
    }
    buf.append(tmp, size_t(k));
    size_t nl;
    while ((nl = buf.find('\n')) != std::string::npos) {
      batch.append(buf, 0, nl + 1);
      buf.erase(0, nl + 1);
      // tracing output may span lines: keep reading until an empty line (spawn.rs:315-326)
      if (tracing_output(batch) && batch.size() >= 2 && batch.compare(batch.size() - 2, 2, "\n\n"))
        continue;
      send_batch(c, batch);
      batch.clear();
    }
  }
  batch += buf;
  if (!batch.empty()) send_batch(c, batch);
  close(rfd);
}

}  // namespace

StdoutCapture* stdout_capture_start(const std::string& output, RequestFn request) {
  auto* c = new StdoutCapture();
  c->output = output;
  c->request = std::move(request);
  int rfd[2] = {-1, -1};
  for (int i = 0; i < 2; ++i) {
    int p[2];
    if (pipe(p) != 0) break;
    rfd[i] = p[0];
    c->wfd[i] = p[1];
    c->saved[i] = dup(i + 1);
  }
  if (rfd[0] < 0 || rfd[1] < 0 || c->saved[0] < 0 || c->saved[1] < 0) {
    for (int i = 0; i < 2; ++i) {
      if (rfd[i] >= 0) close(rfd[i]);
      if (c->wfd[i] >= 0) close(c->wfd[i]);
      if (c->saved[i] >= 0) close(c->saved[i]);
    }
    delete c;
    return nullptr;
  }
  std::fflush(stdout);
  std::fflush(stderr);
  for (int i = 0; i < 2; ++i) {
    dup2(c->wfd[i], i + 1);
    close(c->wfd[i]);
    c->wfd[i] = i + 1;
    c->readers[i] = std::thread(pump, c, rfd[i], c->saved[i]);
  }
  return c;
}

void stdout_capture_stop(StdoutCapture* c) {
  if (!c) return;
  std::fflush(stdout);
  std::fflush(stderr);
  // restoring fd 1 / 2 drops the last write end of each pipe: the readers see EOF
  for (int i = 0; i < 2; ++i) dup2(c->saved[i], i + 1);
  for (auto& t : c->readers)
    if (t.joinable()) t.join();
  for (int i = 0; i < 2; ++i) close(c->saved[i]);
  delete c;
}

}  // namespace dora
