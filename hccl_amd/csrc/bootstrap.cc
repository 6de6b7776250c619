// bootstrap.cc — communicator creation from a rank table file (HcclCommInitClusterInfo) and for all local devices
// (HcclCommInitAll).
//
// Rank table: the JSON cluster description of docs/zh/user_guide/cluster_info_config/rank_table_config_*.md —
// "status" must be "completed"; "server_list"[*]."device"[*] carries "device_id" and "rank_id" (strings or numbers),
// optionally "host_port"; a server may carry "host_ip". rank_id must cover 0 .. N-1 exactly once. The caller's rank runs
// on its entry's device_id (the rank table has priority over the device environment, rank_table_config_a2.md).
//
// RCCL needs one unique id on every rank; a rank table carries no channel for it, so rank 0 publishes it over TCP,
// as HCCL's host-socket bootstrap does: address = the rank-0 server's "host_ip", else HCCL_IF_IP, else 127.0.0.1 for
// a single server; port = the rank-0 device's "host_port", else HCCL_IF_BASE_PORT (default 60000,
// hccl_env/HCCL_IF_BASE_PORT.md); every wait is bounded by HCCL_CONNECT_TIMEOUT (default 120 s) + 20 s
// (hccl_env/HCCL_CONNECT_TIMEOUT.md).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "comm.h"

namespace hccl_amd {

namespace {

// ------------------------------------------------------------------------------------------------ minimal JSON

struct JVal {
    enum Kind { kNull, kBool, kNum, kStr, kArr, kObj } kind = kNull;
    std::string str;  // kStr, and the literal text of a kNum
    std::vector<JVal> arr;
    std::vector<std::pair<std::string, JVal>> obj;

    const JVal* Get(const char* key) const
    {
        if (kind != kObj) return nullptr;
        for (const auto& kv : obj) {
            if (kv.first == key) return &kv.second;
        }
        return nullptr;
    }
};

class JParser {
public:
    JParser(const char* b, const char* e) : p_(b), e_(e) {}

    bool Parse(JVal* out)
    {
        if (!Value(out, 0)) return false;
        Ws();
        return p_ == e_;
    }

private:
    const char* p_;
    const char* e_;

    void Ws()
    {
        while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
    }
    bool Lit(const char* s)
    {
        const size_t n = std::strlen(s);
        if (static_cast<size_t>(e_ - p_) < n || std::strncmp(p_, s, n) != 0) return false;
        p_ += n;
        return true;
    }
    bool Str(std::string* out)
    {
        if (p_ >= e_ || *p_ != '"') return false;
        ++p_;
        out->clear();
        while (p_ < e_ && *p_ != '"') {
            char c = *p_++;
            if (c == '\\') {
                if (p_ >= e_) return false;
                char x = *p_++;
                switch (x) {
                    case 'n': c = '\n'; break;
                    case 't': c = '\t'; break;
                    case 'r': c = '\r'; break;
                    case 'b': c = '\b'; break;
                    case 'f': c = '\f'; break;
                    case 'u': {  // keep ASCII code points, replace the rest (no rank-table field needs them)
                        if (e_ - p_ < 4) return false;
                        const unsigned v = static_cast<unsigned>(std::strtoul(std::string(p_, 4).c_str(), nullptr, 16));
                        p_ += 4;
                        c = v < 0x80 ? static_cast<char>(v) : '?';
                        break;
                    }
                    default: c = x; break;  // \" \\ \/
                }
            }
            out->push_back(c);
        }
        if (p_ >= e_) return false;
        ++p_;
        return true;
    }
    bool Value(JVal* v, int depth)
    {
        if (depth > 64) return false;
        Ws();
        if (p_ >= e_) return false;
        const char c = *p_;
        if (c == '{') {
            ++p_;
            v->kind = JVal::kObj;
            Ws();
            if (p_ < e_ && *p_ == '}') {
                ++p_;
                return true;
            }
            for (;;) {
                Ws();
                std::string k;
                if (!Str(&k)) return false;
                Ws();
                if (p_ >= e_ || *p_ != ':') return false;
                ++p_;
                JVal child;
                if (!Value(&child, depth + 1)) return false;
                v->obj.emplace_back(std::move(k), std::move(child));
                Ws();
                if (p_ < e_ && *p_ == ',') {
                    ++p_;
                    continue;
                }
                if (p_ < e_ && *p_ == '}') {
                    ++p_;
                    return true;
                }
                return false;
            }
        }
        if (c == '[') {
            ++p_;
            v->kind = JVal::kArr;
            Ws();
            if (p_ < e_ && *p_ == ']') {
                ++p_;
                return true;
            }
            for (;;) {
                JVal child;
                if (!Value(&child, depth + 1)) return false;
                v->arr.push_back(std::move(child));
                Ws();
                if (p_ < e_ && *p_ == ',') {
                    ++p_;
                    continue;
                }
                if (p_ < e_ && *p_ == ']') {
                    ++p_;
                    return true;
                }
                return false;
            }
        }
        if (c == '"') {
            v->kind = JVal::kStr;
            return Str(&v->str);
        }
        if (Lit("true") || Lit("false")) {
            v->kind = JVal::kBool;
            return true;
        }
        if (Lit("null")) {
            v->kind = JVal::kNull;
            return true;
        }
        const char* b = p_;
        while (p_ < e_ && (std::strchr("+-0123456789.eE", *p_) != nullptr)) ++p_;
        if (p_ == b) return false;
        v->kind = JVal::kNum;
        v->str.assign(b, p_);
        return true;
    }
};

// A non-negative integer field given as a JSON string ("3") or number (3).
bool UintField(const JVal& o, const char* key, uint64_t* out)
{
    const JVal* v = o.Get(key);
    if (v == nullptr || (v->kind != JVal::kStr && v->kind != JVal::kNum) || v->str.empty()) return false;
    char* end = nullptr;
    const unsigned long long x = std::strtoull(v->str.c_str(), &end, 10);
    if (end == nullptr || *end != '\0' || v->str[0] == '-') return false;
    *out = x;
    return true;
}

std::string StrField(const JVal& o, const char* key)
{
    const JVal* v = o.Get(key);
    return v != nullptr && (v->kind == JVal::kStr || v->kind == JVal::kNum) ? v->str : std::string();
}

// ------------------------------------------------------------------------------------------------ rank table

struct RankEntry {
    int32_t device = -1;
    uint32_t server = 0;  // index into server_list
    int32_t hostPort = -1;
};

struct RankTable {
    std::vector<RankEntry> ranks;  // by rank_id
    std::vector<std::string> serverHostIp;
};

HcclResult LoadRankTable(const char* path, RankTable* rt)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        HCCL_AMD_ERR("rank table %s: cannot open", path);
        return HCCL_E_PARA;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    JVal root;
    JParser parser(text.data(), text.data() + text.size());
    if (!parser.Parse(&root) || root.kind != JVal::kObj) {
        HCCL_AMD_ERR("rank table %s: not valid JSON", path);
        return HCCL_E_PARA;
    }
    if (StrField(root, "status") != "completed") {
        HCCL_AMD_ERR("rank table %s: status is not \"completed\"", path);
        return HCCL_E_PARA;
    }
    const JVal* servers = root.Get("server_list");
    if (servers == nullptr || servers->kind != JVal::kArr || servers->arr.empty()) {
        HCCL_AMD_ERR("rank table %s: no server_list", path);
        return HCCL_E_PARA;
    }
    std::vector<std::pair<uint64_t, RankEntry>> seen;
    for (size_t si = 0; si < servers->arr.size(); ++si) {
        const JVal& srv = servers->arr[si];
        const JVal* devs = srv.Get("device");
        if (srv.kind != JVal::kObj || devs == nullptr || devs->kind != JVal::kArr) {
            HCCL_AMD_ERR("rank table %s: server %zu has no device list", path, si);
            return HCCL_E_PARA;
        }
        rt->serverHostIp.push_back(StrField(srv, "host_ip"));
        for (const JVal& d : devs->arr) {
            uint64_t rank = 0, dev = 0, port = 0;
            if (d.kind != JVal::kObj || !UintField(d, "rank_id", &rank) || !UintField(d, "device_id", &dev)) {
                HCCL_AMD_ERR("rank table %s: a device entry lacks rank_id / device_id", path);
                return HCCL_E_PARA;
            }
            RankEntry e;
            e.device = static_cast<int32_t>(dev);
            e.server = static_cast<uint32_t>(si);
            if (UintField(d, "host_port", &port) && port > 0 && port < 65536) e.hostPort = static_cast<int32_t>(port);
            seen.emplace_back(rank, e);
        }
    }
    const size_t n = seen.size();
    if (n == 0 || n > HCCL_AMD_IR_MAX_SRC) {
        HCCL_AMD_ERR("rank table %s: %zu ranks (1..%d supported)", path, n, HCCL_AMD_IR_MAX_SRC);
        return HCCL_E_PARA;
    }
    rt->ranks.assign(n, RankEntry{});
    std::vector<bool> have(n, false);
    for (const auto& kv : seen) {
        if (kv.first >= n || have[kv.first]) {
            HCCL_AMD_ERR("rank table %s: rank_id %llu out of range or repeated", path, (unsigned long long)kv.first);
            return HCCL_E_PARA;
        }
        have[kv.first] = true;
        rt->ranks[kv.first] = kv.second;
    }
    return HCCL_SUCCESS;
}

// ------------------------------------------------------------------------------------------------ TCP id exchange

constexpr uint32_t kHelloMagic = 0x48434C42;  // "HCLB"

uint64_t EnvU64(const char* name, uint64_t dflt, uint64_t lo, uint64_t hi)
{
    const char* e = std::getenv(name);
    if (e == nullptr || *e == '\0') return dflt;
    char* end = nullptr;
    const unsigned long long v = std::strtoull(e, &end, 10);
    return (end != e && v >= lo && v <= hi) ? v : dflt;
}

bool FullIo(int fd, void* buf, size_t n, bool write, std::chrono::steady_clock::time_point deadline)
{
    char* p = static_cast<char*>(buf);
    while (n != 0) {
        const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline -
                                                                                 std::chrono::steady_clock::now());
        if (left.count() <= 0) return false;
        pollfd pf{fd, static_cast<short>(write ? POLLOUT : POLLIN), 0};
        if (poll(&pf, 1, static_cast<int>(std::min<long long>(left.count(), 1000))) <= 0) continue;
        const ssize_t r = write ? send(fd, p, n, MSG_NOSIGNAL) : recv(fd, p, n, 0);
        if (r <= 0) return false;
        p += r;
        n -= static_cast<size_t>(r);
    }
    return true;
}

HcclResult ResolveRoot(const std::string& host, uint16_t port, sockaddr_storage* sa, socklen_t* len)
{
    addrinfo hints{};
    hints.ai_flags = AI_NUMERICHOST;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || res == nullptr) {
        HCCL_AMD_ERR("bootstrap: root address %s is not a numeric IPv4/IPv6 address", host.c_str());
        return HCCL_E_PARA;
    }
    std::memcpy(sa, res->ai_addr, res->ai_addrlen);
    *len = res->ai_addrlen;
    freeaddrinfo(res);
    return HCCL_SUCCESS;
}

// Rank 0 serves `id` to ranks 1 .. n-1; every other rank fetches it.
HcclResult ExchangeUniqueId(const std::string& host, uint16_t port, uint32_t n, uint32_t rank, char id[128])
{
    if (n == 1) return HCCL_SUCCESS;
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(ConnectTimeoutMs());
    sockaddr_storage sa{};
    socklen_t salen = 0;
    HCCL_CHK(ResolveRoot(host, port, &sa, &salen));
    if (rank == 0) {
        const int ls = socket(sa.ss_family, SOCK_STREAM, 0);
        if (ls < 0) return HCCL_E_TCP_CONNECT;
        const int one = 1;
        (void)setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
        if (bind(ls, reinterpret_cast<sockaddr*>(&sa), salen) != 0 || listen(ls, static_cast<int>(n)) != 0) {
            HCCL_AMD_ERR("bootstrap: cannot listen on %s:%u (%s)", host.c_str(), port, std::strerror(errno));
            close(ls);
            return HCCL_E_TCP_CONNECT;
        }
        // Ranks are counted once each (a rank that retries after a short read is served again, not counted twice),
        // and each connection gets a short deadline of its own, so a stray client that connects and sends nothing
        // holds the accept loop for 2 s, not until HCCL_CONNECT_TIMEOUT.
        std::vector<bool> done(n, false);
        done[0] = true;
        uint32_t served = 0;
        HcclResult r = HCCL_SUCCESS;
        while (served + 1 < n) {
            const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline -
                                                                                     std::chrono::steady_clock::now());
            if (left.count() <= 0) {
                HCCL_AMD_ERR("bootstrap: %u of %u ranks connected before HCCL_CONNECT_TIMEOUT", served + 1, n);
                r = HCCL_E_TIMEOUT;
                break;
            }
            pollfd pf{ls, POLLIN, 0};
            if (poll(&pf, 1, static_cast<int>(std::min<long long>(left.count(), 1000))) <= 0) continue;
            const int cs = accept(ls, nullptr, nullptr);
            if (cs < 0) continue;
            const auto connDeadline = std::min(deadline, std::chrono::steady_clock::now() + std::chrono::seconds(2));
            uint32_t hello[2] = {0, 0};
            if (FullIo(cs, hello, sizeof hello, false, connDeadline) && hello[0] == kHelloMagic && hello[1] < n &&
                hello[1] != 0 && FullIo(cs, id, 128, true, connDeadline) && !done[hello[1]]) {
                done[hello[1]] = true;
                ++served;
            }
            close(cs);
        }
        close(ls);
        return r;
    }
    for (;;) {
        if (std::chrono::steady_clock::now() > deadline) {
            HCCL_AMD_ERR("bootstrap: rank %u could not reach the root at %s:%u before HCCL_CONNECT_TIMEOUT", rank,
                         host.c_str(), port);
            return HCCL_E_TIMEOUT;
        }
        const int s = socket(sa.ss_family, SOCK_STREAM, 0);
        if (s < 0) return HCCL_E_TCP_CONNECT;
        if (connect(s, reinterpret_cast<sockaddr*>(&sa), salen) == 0) {
            const uint32_t hello[2] = {kHelloMagic, rank};
            const bool ok = FullIo(s, const_cast<uint32_t*>(hello), sizeof hello, true, deadline) &&
                            FullIo(s, id, 128, false, deadline);
            close(s);
            if (ok) return HCCL_SUCCESS;
        } else {
            close(s);
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
}

}  // namespace

}  // namespace hccl_amd

using namespace hccl_amd;

extern "C" HcclResult HcclAmdRankTableInfo(const char* clusterInfo, uint32_t rank, uint32_t* nRanks, int32_t* deviceId)
{
    if (clusterInfo == nullptr || nRanks == nullptr || deviceId == nullptr) return HCCL_E_PTR;
    RankTable rt;
    HCCL_CHK(LoadRankTable(clusterInfo, &rt));
    if (rank >= rt.ranks.size()) return HCCL_E_PARA;
    *nRanks = static_cast<uint32_t>(rt.ranks.size());
    *deviceId = rt.ranks[rank].device;
    return HCCL_SUCCESS;
}

namespace hccl_amd {

namespace {

// Where the rank-0 unique id is published for a table: the rank-0 server's host_ip, else HCCL_IF_IP, else 127.0.0.1
// for a single server; the rank-0 device's host_port, else HCCL_IF_BASE_PORT.
HcclResult RootAddress(const RankTable& rt, std::string* host, uint16_t* port)
{
    const RankEntry& root = rt.ranks[0];
    *host = rt.serverHostIp[root.server];
    if (host->empty()) {
        const char* ip = std::getenv("HCCL_IF_IP");
        if (ip != nullptr && *ip != '\0') {
            *host = ip;
        } else if (rt.serverHostIp.size() == 1) {
            *host = "127.0.0.1";
        } else {
            HCCL_AMD_ERR("rank table spans %zu servers: give the rank-0 server a host_ip or set HCCL_IF_IP",
                         rt.serverHostIp.size());
            return HCCL_E_PARA;
        }
    }
    *port = static_cast<uint16_t>(
        root.hostPort > 0 ? static_cast<uint64_t>(root.hostPort) : EnvU64("HCCL_IF_BASE_PORT", 60000, 1024, 65520));
    return HCCL_SUCCESS;
}

HcclResult LoadForRank(const char* clusterInfo, uint32_t rank, RankTable* rt)
{
    HCCL_CHK(LoadRankTable(clusterInfo, rt));
    if (rank >= rt->ranks.size()) {
        HCCL_AMD_ERR("rank %u is not in the rank table (%zu ranks)", rank, rt->ranks.size());
        return HCCL_E_PARA;
    }
    return HCCL_SUCCESS;
}

// The last HcclCommInitClusterInfo of the process (HcclAmdLastBootstrap).
std::atomic<uint64_t> gLastIdDigest{0};
std::atomic<int32_t> gLastStage{0};

uint64_t Fnv1a64(const char* p, size_t n)
{
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) {
        h ^= static_cast<uint8_t>(p[i]);
        h *= 1099511628211ull;
    }
    return h;
}

}  // namespace

}  // namespace hccl_amd

extern "C" HcclResult HcclAmdBootstrapExchangeId(const char* clusterInfo, uint32_t rank, void* id128)
{
    if (clusterInfo == nullptr || id128 == nullptr) return HCCL_E_PTR;
    RankTable rt;
    HCCL_CHK(LoadForRank(clusterInfo, rank, &rt));
    std::string host;
    uint16_t port = 0;
    HCCL_CHK(RootAddress(rt, &host, &port));
    return ExchangeUniqueId(host, port, static_cast<uint32_t>(rt.ranks.size()), rank, static_cast<char*>(id128));
}

extern "C" HcclResult HcclAmdLastBootstrap(uint64_t* idDigest, int32_t* stage)
{
    if (idDigest == nullptr || stage == nullptr) return HCCL_E_PTR;
    *stage = gLastStage.load();
    *idDigest = gLastIdDigest.load();
    return HCCL_SUCCESS;
}

extern "C" HcclResult HcclCommInitClusterInfo(const char* clusterInfo, uint32_t rank, HcclComm* comm)
{
    if (clusterInfo == nullptr || comm == nullptr) return HCCL_E_PTR;
    gLastStage = 0;
    gLastIdDigest = 0;
    RankTable rt;
    HCCL_CHK(LoadForRank(clusterInfo, rank, &rt));
    const uint32_t n = static_cast<uint32_t>(rt.ranks.size());
    std::string host;
    uint16_t port = 0;
    HCCL_CHK(RootAddress(rt, &host, &port));
    HIP_CHK(hipSetDevice(rt.ranks[rank].device));
    char id[128] = {};
    if (rank == 0) HCCL_CHK(RcclGetUniqueId(id));
    HCCL_CHK(ExchangeUniqueId(host, port, n, rank, id));
    gLastIdDigest = Fnv1a64(id, sizeof id);
    gLastStage = 1;
    auto c = std::make_unique<Comm>();
    c->rank = rank;
    c->nRanks = n;
    HCCL_CHK(c->Init(rt.ranks[rank].device));
    HcclResult err = HCCL_SUCCESS;
    c->transport = MakeRcclTransport(id, n, rank, &err);
    if (c->transport == nullptr) return err == HCCL_SUCCESS ? HCCL_E_INTERNAL : err;
    HCCL_CHK(c->StartWatchdog());
    gLastStage = 2;
    *comm = c.release();
    return HCCL_SUCCESS;
}

extern "C" HcclResult HcclCommInitAll(uint32_t ndev, int32_t* devices, HcclComm* comms)
{
    if (devices == nullptr || comms == nullptr) return HCCL_E_PTR;
    if (ndev == 0 || ndev > HCCL_AMD_IR_MAX_SRC) return HCCL_E_PARA;
    int count = 0;
    HIP_CHK(hipGetDeviceCount(&count));
    for (uint32_t i = 0; i < ndev; ++i) {
        if (devices[i] < 0 || devices[i] >= count) return HCCL_E_PARA;
        for (uint32_t j = 0; j < i; ++j) {
            if (devices[j] == devices[i]) return HCCL_E_PARA;  // one rank per device
        }
    }
    std::vector<std::unique_ptr<Comm>> made(ndev);
    for (uint32_t r = 0; r < ndev; ++r) {
        made[r] = std::make_unique<Comm>();
        made[r]->rank = r;
        made[r]->nRanks = ndev;
        HIP_CHK(hipSetDevice(devices[r]));
        HCCL_CHK(made[r]->Init(devices[r]));
    }
    std::vector<std::unique_ptr<Transport>> transports;
    HCCL_CHK(MakeRcclTransportsAll(ndev, devices, &transports));
    for (uint32_t r = 0; r < ndev; ++r) {
        made[r]->transport = std::move(transports[r]);
        HCCL_CHK(made[r]->StartWatchdog());
    }
    for (uint32_t r = 0; r < ndev; ++r) comms[r] = made[r].release();
    return HCCL_SUCCESS;
}
