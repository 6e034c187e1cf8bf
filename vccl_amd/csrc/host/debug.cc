// Logging and environment parameters.
// Reference idioms: NCCL_DEBUG / ncclDebugLog (src/debug.cc, include/debug.h:22-34)
// and NCCL_PARAM (include/param.h:17-25, misc/param.cc:52-98).
#include <atomic>
#include <cstdarg>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unistd.h>

#include "core.h"

namespace vccl {

static int parse_level(const char* s) {
  if (!s) return kLogWarn;
  if (!strcasecmp(s, "VERSION") || !strcasecmp(s, "WARN")) return kLogWarn;
  if (!strcasecmp(s, "INFO")) return kLogInfo;
  if (!strcasecmp(s, "TRACE")) return kLogTrace;
  if (!strcasecmp(s, "NONE")) return kLogNone;
  return kLogWarn;
}

// -1: not read yet (first use, or after ncclResetDebugInit)
static std::atomic<int> g_level{-1};

// NCCL_DEBUG_SUBSYS (debug.cc:57-111): which subsystems' INFO lines print;
// the reference's default is INIT, BOOTSTRAP and ENV (debug.cc:30), so the
// per-call COLL trace needs NCCL_DEBUG_SUBSYS=COLL as with libnccl.  WARNs
// always print.  A line's subsystem is its source file's.
enum : uint64_t {
  kSubInit = 1, kSubColl = 2, kSubP2P = 4, kSubShm = 8, kSubNet = 16, kSubGraph = 32,
  kSubTuning = 64, kSubEnv = 128, kSubAlloc = 256, kSubCall = 512, kSubProxy = 1024,
  kSubNvls = 2048, kSubBootstrap = 4096, kSubReg = 8192, kSubProfile = 16384, kSubRas = 32768,
  kSubDefault = kSubInit | kSubBootstrap | kSubEnv
};
static std::atomic<uint64_t> g_mask{kSubDefault};

static uint64_t debug_subsys_mask(const char* spec) {
  if (!spec) return kSubDefault;
  static const struct { const char* name; uint64_t bit; } kNames[] = {
      {"INIT", kSubInit}, {"COLL", kSubColl}, {"P2P", kSubP2P}, {"SHM", kSubShm}, {"NET", kSubNet},
      {"GRAPH", kSubGraph}, {"TUNING", kSubTuning}, {"ENV", kSubEnv}, {"ALLOC", kSubAlloc},
      {"CALL", kSubCall}, {"PROXY", kSubProxy}, {"NVLS", kSubNvls}, {"BOOTSTRAP", kSubBootstrap},
      {"REG", kSubReg}, {"PROFILE", kSubProfile}, {"RAS", kSubRas}, {"ALL", ~0ull}};
  const bool invert = spec[0] == '^';
  uint64_t mask = invert ? ~0ull : 0;
  std::string list(spec + (invert ? 1 : 0));
  size_t at = 0;
  while (at <= list.size()) {
    size_t end = list.find(',', at);
    if (end == std::string::npos) end = list.size();
    const std::string item = list.substr(at, end - at);
    for (const auto& n : kNames)
      if (!strcasecmp(item.c_str(), n.name)) mask = invert ? mask & ~n.bit : mask | n.bit;
    at = end + 1;
  }
  return mask;
}

static uint64_t subsys_of(const char* base) {
  if (!strncmp(base, "enqueue", 7)) return kSubColl;
  if (!strncmp(base, "proxy", 5)) return kSubNet | kSubProxy;
  if (!strncmp(base, "bootstrap", 9)) return kSubBootstrap;
  if (!strncmp(base, "debug", 5)) return kSubEnv;
  return kSubInit;
}

// NCCL_DEBUG_FILE (debug.cc:209-255): the log's file, else stderr.  g_initMu
// guards the first read of the environment; log_msg holds g_mu while it
// writes and may then take g_initMu, so every path takes g_mu first.
static std::mutex g_initMu;
static std::mutex g_mu;
static std::atomic<FILE*> g_file{nullptr};

// The file name of NCCL_DEBUG_FILE: %h the host name, %p the pid, %% a
// '%', any other %-sequence kept as written (debug.cc:215-247).
static std::string debug_file_name(const char* pattern, const char* host, int pid) {
  std::string out;
  for (const char* c = pattern; *c; c++) {
    if (*c != '%') {
      out += *c;
      continue;
    }
    const char k = *++c;
    if (k == '%') out += '%';
    else if (k == 'h') out += host;
    else if (k == 'p') out += std::to_string(pid);
    else {
      out += '%';
      if (!k) break;
      out += k;
    }
  }
  return out;
}

int log_level() {
  int level = g_level.load(std::memory_order_acquire);
  if (level >= 0) return level;
  std::lock_guard<std::mutex> lk(g_initMu);
  level = g_level.load(std::memory_order_relaxed);
  if (level >= 0) return level;
  const char* s = getenv("VCCL_DEBUG");
  if (!s) s = getenv("NCCL_DEBUG");
  level = parse_level(s);
  const char* sub = getenv("VCCL_DEBUG_SUBSYS");
  if (!sub) sub = getenv("NCCL_DEBUG_SUBSYS");
  g_mask.store(debug_subsys_mask(sub), std::memory_order_relaxed);
  // as the reference: only for an explicit level above VERSION
  const char* f = getenv("VCCL_DEBUG_FILE");
  if (!f) f = getenv("NCCL_DEBUG_FILE");
  if (f && s && level >= kLogWarn && strcasecmp(s, "VERSION") != 0 && !g_file.load()) {
    char host[256] = "";
    gethostname(host, sizeof(host) - 1);
    if (char* dot = strchr(host, '.')) *dot = '\0';  // getHostName(..., '.')
    const std::string name = debug_file_name(f, host, (int)getpid());
    if (!name.empty()) {
      if (FILE* fp = fopen(name.c_str(), "w")) {
        setbuf(fp, nullptr);  // unbuffered, as the reference
        g_file.store(fp);
      }
    }
  }
  g_level.store(level, std::memory_order_release);
  return level;
}

// ncclResetDebugInit (debug.cc:367-378): the next log call re-reads the
// level, and the debug file is closed
void reset_log_level() {
  std::lock_guard<std::mutex> lk(g_mu);
  std::lock_guard<std::mutex> li(g_initMu);
  if (FILE* fp = g_file.exchange(nullptr)) fclose(fp);
  g_level.store(-1, std::memory_order_release);
}

// ncclLastError (debug.cc:29): the last WARN as human-readable text, saved
// before the level filter (debug.cc:265-272), returned by ncclGetLastError.
static char g_lastError[1024] = "";
const char* last_error() { return g_lastError; }

void log_msg(int level, const char* file, int line, const char* fmt, ...) {
  const bool warn = level == kLogWarn;
  if (!warn && log_level() < level) return;
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> lk(g_mu);
  if (warn) memcpy(g_lastError, buf, sizeof(buf));
  if (log_level() < level) return;
  const char* base = strrchr(file, '/');
  base = base ? base + 1 : file;
  if (!warn && !(subsys_of(base) & g_mask.load(std::memory_order_relaxed))) return;
  FILE* out = g_file.load();
  fprintf(out ? out : stderr, "[vccl %d] %s %s:%d %s\n", (int)getpid(),
          level == kLogWarn ? "WARN" : "INFO", base, line, buf);
}

int64_t param_int(const char* name, int64_t deflt) {
  char key[128];
  snprintf(key, sizeof(key), "VCCL_%s", name);
  const char* s = getenv(key);
  if (!s) {
    snprintf(key, sizeof(key), "NCCL_%s", name);
    s = getenv(key);
  }
  if (!s || !*s) return deflt;
  char* end = nullptr;
  long long v = strtoll(s, &end, 0);
  if (end == s) {
    VWARN("invalid value '%s' for %s, using %lld", s, key, (long long)deflt);
    return deflt;
  }
  return v;
}

}  // namespace vccl
