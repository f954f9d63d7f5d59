// kfamd-launch: per-node launcher / rendezvous / health agent for one-process-per-GPU jobs
// on MI355X nodes (SURVEY.md §1.2 layer D3, §3.7).
//
// What the PyTorchJob / MPIJob operators put in a pod is:
//   kfamd-launch --nnodes N|MIN:MAX --node-rank R --nproc-per-node P \
//                --master-addr A --master-port M [--rdzv-port Q] [--max-restarts K] \
//                [--rdzv-last-call S] [--heartbeat-timeout S] [--isolate-devices] -- <worker command...>
//
// 1. Rendezvous (TCP, node 0 hosts it on --rdzv-port, default M+1): every node agent
//    registers (node_rank, nproc, hostname); once all N have joined, the server sends each
//    agent its global rank offset, the world size and a round id.  A restart starts a new
//    round, so all nodes restart their workers together.
//    Elastic (--nnodes MIN:MAX, PyTorchJob elasticPolicy): a round closes when MAX agents
//    have joined, or when at least MIN have and no new one has joined for --rdzv-last-call
//    seconds -- and never without node 0: its local rank 0 is global rank 0, which hosts the
//    TCPStore at MASTER_ADDR:MASTER_PORT, so a round without it would be a second world
//    pointed at the running one's store.  Rank offsets follow node-rank order among the
//    members, so after a node is lost the survivors' restart re-forms the group at the
//    smaller world size.
//    Membership changes (torchrun's "nodes waiting" rule): while its workers run, every agent
//    of a multi-node job polls the server about once a second; as soon as any agent has
//    joined the NEXT round (a replacement pod, a late node, or a member whose workers failed)
//    the running agents stop their workers and re-join, without using up a --max-restarts
//    attempt.  A replacement node is thereby admitted at once instead of after the running
//    group's collectives time out.
//    Node 0 hosts the rendezvous server: if its pod is lost the survivors' workers fail (rank
//    0 and its store are gone) and their agents wait up to --rdzv-timeout for node 0 to come
//    back; a replacement node-0 pod (restartPolicy OnFailure / ExitCode) starts a new server
//    and the job continues, with restartPolicy Never the survivors exit 3 after the timeout.
// 2. Spawn: P workers per node, each with RANK, LOCAL_RANK, WORLD_SIZE,
//    LOCAL_WORLD_SIZE, GROUP_RANK, NODE_RANK, MASTER_ADDR, MASTER_PORT (and the OpenMPI
//    OMPI_COMM_WORLD_{RANK,SIZE,LOCAL_RANK,LOCAL_SIZE} names), the ROCm IPC
//    setting HSA_ENABLE_IPC_MODE_LEGACY=0 (dmabuf IPC for RCCL / tensor sharing) and
//    TORCH_NCCL_ASYNC_ERROR_HANDLING=1 (RCCL async error -> abort, so a hung/failed
//    collective surfaces as a process exit).  With --isolate-devices each worker gets
//    exactly one GPU in HIP_VISIBLE_DEVICES (taken from the pod's device-plugin list).
//    Rank 0 hosts torch.distributed's TCPStore at MASTER_ADDR:MASTER_PORT, through which
//    RCCL's unique id is exchanged.
// 3. Health: any worker exiting non-zero, or any worker missing its heartbeat deadline
//    (worker touches $KFAMD_HEARTBEAT_FILE every step; --heartbeat-timeout S), fails the
//    group: the rest get SIGTERM, then SIGKILL after a grace period.  With restarts left
//    the agent re-rendezvouses and relaunches; otherwise it exits with the failing code.
//
// Pure POSIX C++17 -- no ROCm dependency, so it builds and is tested on CPU hosts.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Args {
  int nnodes = 1, node_rank = 0, nproc = 1, max_restarts = 0;
  int min_nodes = 1;                       // elastic lower bound (== nnodes unless MIN:MAX)
  double last_call = 5.0;                  // elastic: quiet period before a round closes at >= MIN
  std::string master_addr = "127.0.0.1";
  int master_port = 29500, rdzv_port = -1;
  double heartbeat_timeout = 0.0, rdzv_timeout = 600.0, grace = 10.0;
  bool isolate = false;
  std::vector<std::string> cmd;
};

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

void logf(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::fprintf(stderr, "[kfamd-launch] ");
  std::vfprintf(stderr, fmt, ap);
  std::fprintf(stderr, "\n");
  va_end(ap);
}

[[noreturn]] void usage() {
  std::fprintf(stderr,
               "usage: kfamd-launch [--nnodes N] [--node-rank R] [--nproc-per-node P]\n"
               "  [--master-addr A] [--master-port M] [--rdzv-port Q] [--max-restarts K]\n"
               "  [--rdzv-last-call S] [--heartbeat-timeout S] [--rdzv-timeout S] [--isolate-devices] -- cmd...\n"
               "  --nnodes MIN:MAX = elastic membership (PET_NNODES / PET_RDZV_ENDPOINT / PET_MAX_RESTARTS too)\n");
  std::exit(2);
}

// "N" or "MIN:MAX"
void parse_nnodes(const std::string& v, Args& a) {
  const size_t c = v.find(':');
  if (c == std::string::npos) {
    a.nnodes = a.min_nodes = std::stoi(v);
  } else {
    a.min_nodes = std::stoi(v.substr(0, c));
    a.nnodes = std::stoi(v.substr(c + 1));
  }
}

Args parse(int argc, char** argv) {
  Args a;
  auto env_int = [](const char* k, int d) { const char* v = getenv(k); return v ? atoi(v) : d; };
  // operator-injected defaults (training-operator PET_* convention)
  parse_nnodes(getenv("PET_NNODES") ? getenv("PET_NNODES") : "1", a);
  a.node_rank = env_int("PET_NODE_RANK", 0);
  a.nproc = env_int("PET_NPROC_PER_NODE", 1);
  a.max_restarts = env_int("PET_MAX_RESTARTS", 0);
  if (const char* v = getenv("PET_MASTER_ADDR")) a.master_addr = v;
  a.master_port = env_int("PET_MASTER_PORT", 29500);
  if (const char* v = getenv("PET_RDZV_ENDPOINT")) {          // host:port of the c10d-style rendezvous
    const std::string e = v;
    const size_t c = e.rfind(':');
    if (c != std::string::npos) a.rdzv_port = std::stoi(e.substr(c + 1));
  }
  if (const char* v = getenv("KFAMD_RDZV_LAST_CALL")) a.last_call = std::stod(v);
  if (const char* v = getenv("KFAMD_RDZV_TIMEOUT")) a.rdzv_timeout = std::stod(v);
  int i = 1;
  for (; i < argc; ++i) {
    std::string s = argv[i];
    auto next = [&]() -> std::string { if (i + 1 >= argc) usage(); return argv[++i]; };
    if (s == "--") { ++i; break; }
    else if (s == "--nnodes") parse_nnodes(next(), a);
    else if (s == "--rdzv-last-call") a.last_call = std::stod(next());
    else if (s == "--node-rank") a.node_rank = std::stoi(next());
    else if (s == "--nproc-per-node") a.nproc = std::stoi(next());
    else if (s == "--master-addr") a.master_addr = next();
    else if (s == "--master-port") a.master_port = std::stoi(next());
    else if (s == "--rdzv-port") a.rdzv_port = std::stoi(next());
    else if (s == "--max-restarts") a.max_restarts = std::stoi(next());
    else if (s == "--heartbeat-timeout") a.heartbeat_timeout = std::stod(next());
    else if (s == "--rdzv-timeout") a.rdzv_timeout = std::stod(next());
    else if (s == "--grace") a.grace = std::stod(next());
    else if (s == "--isolate-devices") a.isolate = true;
    else if (s == "-h" || s == "--help") usage();
    else { a.cmd.push_back(s); }
  }
  for (; i < argc; ++i) a.cmd.push_back(argv[i]);
  if (a.cmd.empty() || a.nnodes < 1 || a.min_nodes < 1 || a.min_nodes > a.nnodes || a.nproc < 1 ||
      a.node_rank < 0 || a.node_rank >= a.nnodes)
    usage();
  if (a.rdzv_port < 0) a.rdzv_port = a.master_port + 1;
  return a;
}

// ------------------------------------------------------------------ line-based TCP helpers
bool send_line(int fd, const std::string& s) {
  std::string m = s + "\n";
  size_t off = 0;
  while (off < m.size()) {
    ssize_t n = ::send(fd, m.data() + off, m.size() - off, MSG_NOSIGNAL);
    if (n <= 0) return false;
    off += (size_t)n;
  }
  return true;
}

bool recv_line(int fd, std::string& out, double timeout_s) {
  out.clear();
  double deadline = now_s() + timeout_s;
  char c;
  while (true) {
    if (now_s() > deadline) return false;
    timeval tv{0, 200000};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    ssize_t n = ::recv(fd, &c, 1, 0);
    if (n == 1) {
      if (c == '\n') return true;
      out.push_back(c);
    } else if (n == 0) {
      return false;
    } else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
      return false;
    }
    if (g_stop) return false;
  }
}

int listen_on(int port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr.s_addr = htonl(INADDR_ANY);
  sa.sin_port = htons((uint16_t)port);
  if (::bind(fd, (sockaddr*)&sa, sizeof sa) != 0 || ::listen(fd, 256) != 0) {
    logf("cannot listen on port %d: %s", port, strerror(errno));
    ::close(fd);
    return -1;
  }
  return fd;
}

int connect_to(const std::string& host, int port, double timeout_s) {
  double deadline = now_s() + timeout_s;
  while (now_s() < deadline && !g_stop) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res) {
      int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        return fd;
      }
      ::close(fd);
      freeaddrinfo(res);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
  }
  return -1;
}

// ------------------------------------------------------------------ rendezvous
struct Assignment {
  int rank_offset = 0, world = 0, round = 0;
};

// Node 0: serve one rendezvous round (all nnodes join) and answer every member.
// Runs in a background thread for the launcher's lifetime so restarts can re-join.
struct RdzvServer {
  int fd = -1, nnodes = 1, min_nodes = 1;
  double last_call = 5.0, grace = 10.0;
  std::thread th;
  void start(int port, int nn, int mn, double lc, double gr) {
    nnodes = nn;
    min_nodes = mn;
    last_call = lc;
    grace = gr;
    fd = listen_on(port);
    if (fd < 0) return;
    th = std::thread([this] { loop(); });
    th.detach();
  }
  // a round is complete with all nnodes members, or (elastic) with >= min_nodes and no join
  // for last_call seconds; never without node 0 (global rank 0 and its store live there).
  // The early (elastic) close also waits for every member of the previous round, for up to
  // grace + last_call after this round's first JOIN: on a membership change each running agent
  // stops its workers (SIGTERM, up to --grace seconds) BEFORE it re-joins, so a node whose
  // workers exit slowly must not be closed out of the round it is about to join.
  bool complete(const std::map<int, std::pair<int, int>>& m, double last_join, double first_join,
                const std::set<int>& prev) const {
    if (!m.count(0)) return false;
    if ((int)m.size() >= nnodes) return true;
    if (!((int)m.size() >= min_nodes && min_nodes < nnodes && now_s() - last_join >= last_call)) return false;
    for (int p : prev)
      if (!m.count(p)) return first_join >= 0 && now_s() - first_join >= grace + last_call;
    return true;
  }
  void loop() {
    int round = 0;
    std::set<int> prev;                            // node ranks of the last closed round
    while (!g_stop) {
      std::map<int, std::pair<int, int>> members;  // node_rank -> (nproc, fd)
      double last_join = now_s(), first_join = -1;
      while (!complete(members, last_join, first_join, prev) && !g_stop) {
        pollfd pfd{fd, POLLIN, 0};
        if (::poll(&pfd, 1, 100) <= 0) continue;
        int c = ::accept(fd, nullptr, nullptr);
        if (c < 0) continue;
        std::string line;
        if (!recv_line(c, line, 30.0)) { ::close(c); continue; }
        std::istringstream is(line);
        std::string tag;
        int nr = -1, np = 0;
        is >> tag >> nr >> np;
        if (tag == "POLL") {
          // a running agent asks whether to restart: agents waiting for the next round, and the
          // last round closed (an agent of an older round is stale and must re-join too)
          send_line(c, "WAIT " + std::to_string(members.size()) + " " + std::to_string(round));
          ::close(c);
          continue;
        }
        if (tag != "JOIN" || nr < 0 || nr >= nnodes || np < 1) { send_line(c, "ERR bad join"); ::close(c); continue; }
        if (members.count(nr)) ::close(members[nr].second);   // a restarted agent re-joins
        members[nr] = {np, c};
        last_join = now_s();
        if (first_join < 0) first_join = last_join;
      }
      if (g_stop) break;
      ++round;
      prev.clear();
      for (auto& m : members) prev.insert(m.first);
      int offset = 0, world = 0;
      for (auto& m : members) world += m.second.first;
      for (auto& m : members) {
        send_line(m.second.second, "OK " + std::to_string(offset) + " " + std::to_string(world) + " " +
                                       std::to_string(round));
        offset += m.second.first;
        ::close(m.second.second);
      }
    }
  }
};

bool rendezvous(const Args& a, Assignment& out) {
  int fd = connect_to(a.node_rank == 0 ? "127.0.0.1" : a.master_addr, a.rdzv_port, a.rdzv_timeout);
  if (fd < 0) { logf("rendezvous: cannot reach %s:%d", a.master_addr.c_str(), a.rdzv_port); return false; }
  send_line(fd, "JOIN " + std::to_string(a.node_rank) + " " + std::to_string(a.nproc));
  std::string line;
  bool ok = recv_line(fd, line, a.rdzv_timeout);
  ::close(fd);
  if (!ok) { logf("rendezvous: timed out waiting for %d nodes", a.min_nodes); return false; }
  std::istringstream is(line);
  std::string tag;
  is >> tag >> out.rank_offset >> out.world >> out.round;
  return tag == "OK";
}

// Running agent: should this round's workers stop so the agent can re-join?  True when another
// agent waits for the next round or a newer round has closed.  An unreachable server (node 0
// lost) says nothing: the workers find out through their collectives.
bool membership_changed(const Args& a, int my_round) {
  int fd = connect_to(a.node_rank == 0 ? "127.0.0.1" : a.master_addr, a.rdzv_port, 1.0);
  if (fd < 0) return false;
  send_line(fd, "POLL " + std::to_string(a.node_rank) + " " + std::to_string(my_round));
  std::string line;
  const bool ok = recv_line(fd, line, 2.0);
  ::close(fd);
  if (!ok) return false;
  std::istringstream is(line);
  std::string tag;
  int waiting = 0, closed = 0;
  is >> tag >> waiting >> closed;
  return tag == "WAIT" && (waiting > 0 || closed > my_round);
}

// ------------------------------------------------------------------ workers
std::vector<std::string> split(const std::string& s, char d) {
  std::vector<std::string> v;
  std::string cur;
  for (char c : s) { if (c == d) { v.push_back(cur); cur.clear(); } else cur.push_back(c); }
  if (!cur.empty()) v.push_back(cur);
  return v;
}

struct Worker {
  pid_t pid = -1;
  int local_rank = 0;
  std::string hb_file;
  int status = 0;
  bool done = false;
};

pid_t spawn(const Args& a, const Assignment& as, int lr, const std::string& hb) {
  pid_t pid = fork();
  if (pid != 0) return pid;
  setpgid(0, 0);
  auto set = [](const char* k, const std::string& v) { setenv(k, v.c_str(), 1); };
  set("RANK", std::to_string(as.rank_offset + lr));
  set("LOCAL_RANK", std::to_string(lr));
  set("WORLD_SIZE", std::to_string(as.world));
  set("LOCAL_WORLD_SIZE", std::to_string(a.nproc));
  set("GROUP_RANK", std::to_string(a.node_rank));
  set("NODE_RANK", std::to_string(a.node_rank));
  set("MASTER_ADDR", a.master_addr);
  set("MASTER_PORT", std::to_string(a.master_port));
  set("KFAMD_RDZV_ROUND", std::to_string(as.round));
  // the OpenMPI names too, for programs written against mpirun's environment (MPIJob workers)
  set("OMPI_COMM_WORLD_RANK", std::to_string(as.rank_offset + lr));
  set("OMPI_COMM_WORLD_SIZE", std::to_string(as.world));
  set("OMPI_COMM_WORLD_LOCAL_RANK", std::to_string(lr));
  set("OMPI_COMM_WORLD_LOCAL_SIZE", std::to_string(a.nproc));
  set("HSA_ENABLE_IPC_MODE_LEGACY", "0");
  set("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1");
  if (!hb.empty()) set("KFAMD_HEARTBEAT_FILE", hb);
  if (a.isolate) {
    const char* vis = getenv("HIP_VISIBLE_DEVICES");
    std::vector<std::string> ids = vis ? split(vis, ',') : std::vector<std::string>{};
    std::string mine = lr < (int)ids.size() ? ids[lr] : std::to_string(lr);
    set("HIP_VISIBLE_DEVICES", mine);
    set("LOCAL_RANK", "0");
    set("KFAMD_LOCAL_RANK", std::to_string(lr));
  }
  std::vector<char*> argv;
  for (auto& s : a.cmd) argv.push_back(const_cast<char*>(s.c_str()));
  argv.push_back(nullptr);
  execvp(argv[0], argv.data());
  std::perror("execvp");
  _exit(127);
}

double mtime(const std::string& f) {
  struct stat st;
  if (stat(f.c_str(), &st) != 0) return -1;
  return (double)st.st_mtim.tv_sec + st.st_mtim.tv_nsec * 1e-9;
}

void kill_all(std::vector<Worker>& ws, double grace) {
  for (auto& w : ws)
    if (!w.done && w.pid > 0) kill(-w.pid, SIGTERM);
  double deadline = now_s() + grace;
  while (now_s() < deadline) {
    bool any = false;
    for (auto& w : ws) {
      if (w.done) continue;
      int st;
      if (waitpid(w.pid, &st, WNOHANG) == w.pid) { w.done = true; w.status = st; }
      else any = true;
    }
    if (!any) return;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  for (auto& w : ws)
    if (!w.done) { kill(-w.pid, SIGKILL); waitpid(w.pid, &w.status, 0); w.done = true; }
}

int exit_code(int st) {
  if (WIFEXITED(st)) return WEXITSTATUS(st);
  if (WIFSIGNALED(st)) return 128 + WTERMSIG(st);
  return 1;
}

constexpr int kMembershipChange = -1;

// run one round; returns 0 on success, kMembershipChange when the agent must re-join for a
// membership change, else the failing exit code
int run_round(const Args& a, const Assignment& as) {
  std::vector<Worker> ws(a.nproc);
  char tmpl[] = "/tmp/kfamd-hb-XXXXXX";
  std::string hbdir;
  if (a.heartbeat_timeout > 0 && mkdtemp(tmpl)) hbdir = tmpl;
  double t0 = now_s();
  for (int lr = 0; lr < a.nproc; ++lr) {
    ws[lr].local_rank = lr;
    if (!hbdir.empty()) ws[lr].hb_file = hbdir + "/rank" + std::to_string(lr);
    ws[lr].pid = spawn(a, as, lr, ws[lr].hb_file);
  }
  logf("round %d: started %d workers (ranks %d..%d of %d)", as.round, a.nproc, as.rank_offset,
       as.rank_offset + a.nproc - 1, as.world);
  int rc = 0;
  double next_poll = now_s() + 1.0;
  while (true) {
    if (g_stop) { kill_all(ws, a.grace); rc = 143; break; }
    if (a.nnodes > 1 && now_s() >= next_poll) {
      next_poll = now_s() + 1.0;
      if (membership_changed(a, as.round)) {
        logf("round %d: membership change (an agent is waiting for the next round): restarting workers",
             as.round);
        kill_all(ws, a.grace);
        rc = kMembershipChange;
        break;
      }
    }
    bool all_done = true, failed = false;
    for (auto& w : ws) {
      if (w.done) continue;
      int st;
      pid_t r = waitpid(w.pid, &st, WNOHANG);
      if (r == w.pid) {
        w.done = true;
        w.status = st;
        if (exit_code(st) != 0) {
          logf("worker local_rank=%d exited with code %d", w.local_rank, exit_code(st));
          rc = exit_code(st);
          failed = true;
        }
      } else {
        all_done = false;
        if (a.heartbeat_timeout > 0) {
          double m = mtime(w.hb_file);
          double last = m < 0 ? t0 : m;
          double wall = (double)std::chrono::duration<double>(
                            std::chrono::system_clock::now().time_since_epoch()).count();
          // before the first heartbeat, allow startup time of 4x the timeout
          double limit = m < 0 ? 4 * a.heartbeat_timeout : a.heartbeat_timeout;
          double age = m < 0 ? now_s() - last : wall - last;
          if (age > limit) {
            logf("worker local_rank=%d missed its heartbeat (%.1fs > %.1fs): treating as hung",
                 w.local_rank, age, limit);
            rc = 124;
            failed = true;
          }
        }
      }
    }
    if (failed) { kill_all(ws, a.grace); break; }
    if (all_done) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  if (!hbdir.empty()) {
    for (auto& w : ws) unlink(w.hb_file.c_str());
    rmdir(hbdir.c_str());
  }
  return rc;
}

}  // namespace

int main(int argc, char** argv) {
  Args a = parse(argc, argv);
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  signal(SIGPIPE, SIG_IGN);
  RdzvServer server;
  if (a.node_rank == 0) server.start(a.rdzv_port, a.nnodes, a.min_nodes, a.last_call, a.grace);
  int rc = 1;
  for (int attempt = 0; attempt <= a.max_restarts;) {
    Assignment as;
    if (!rendezvous(a, as)) { rc = 3; break; }
    rc = run_round(a, as);
    if (rc == 0 || g_stop) break;
    if (rc == kMembershipChange) { rc = 1; continue; }   // not a failure: no restart used
    if (attempt < a.max_restarts) logf("restarting workers (%d of %d restarts used)", attempt + 1, a.max_restarts);
    ++attempt;
  }
  logf("exit %d", rc);
  return rc;
}
