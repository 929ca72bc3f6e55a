// minisched.cpp — see minisched.h. Citations are into /root/reference.
#include "minisched.h"

#include <algorithm>
#include <stdexcept>

namespace minisched {

// ------------------------------------------------------------------------ v1
namespace v1 {

bool Toleration::ToleratesTaint(const Taint &t) const {
    if (!effect.empty() && effect != t.effect) return false;
    if (!key.empty() && key != t.key) return false;
    if (op.empty() || op == "Equal") return value == t.value;  // empty operator means Equal
    if (op == "Exists") return true;
    return false;
}

bool TolerationsTolerateTaint(const std::vector<Toleration> &tols, const Taint &t) {
    for (const auto &x : tols)
        if (x.ToleratesTaint(t)) return true;
    return false;
}

}  // namespace v1

// ------------------------------------------------------------------- plugins
using framework::ClusterEvent;

std::vector<ClusterEvent> NodeUnschedulable::EventsToRegister() const {
    return {{framework::kNode, framework::Add | framework::UpdateNodeTaint, ""}};
}
std::vector<ClusterEvent> NodeNumber::EventsToRegister() const {
    return {{framework::kNode, framework::Add, ""}};  // nodenumber.go:66-70
}
std::vector<ClusterEvent> NodeResourcesFit::EventsToRegister() const {
    return {{framework::kPod, framework::Delete, ""},
            {framework::kNode, framework::Add | framework::UpdateNodeAllocatable, ""}};
}

// --------------------------------------------------------------------- queue
SchedulingQueue::SchedulingQueue(std::map<ClusterEvent, std::set<std::string>> m, Clock clock)
    : event_map_(std::move(m)), clock_(std::move(clock)) {}

std::chrono::steady_clock::time_point SchedulingQueue::Now() const {
    return clock_ ? clock_() : std::chrono::steady_clock::now();
}

void SchedulingQueue::Add(const v1::Pod &pod) {  // queue.go:35-43 + newQueuedPodInfo :158-166
    framework::QueuedPodInfo p;
    p.pod = pod;
    p.timestamp = p.initial_attempt_timestamp = Now();
    active_.push_back(std::move(p));
}

std::optional<v1::Pod> SchedulingQueue::NextPod() {  // queue.go:84-92 without the busy spin
    if (active_.empty()) return std::nullopt;
    v1::Pod p = std::move(active_.front().pod);
    active_.pop_front();
    return p;
}

void SchedulingQueue::AddUnschedulable(framework::QueuedPodInfo pinfo) {  // queue.go:95-107
    pinfo.timestamp = Now();  // "Refresh the timestamp since the pod is re-added."
    const std::string k = KeyFunc(pinfo.pod);
    unschedulable_[k] = std::move(pinfo);
}

const framework::QueuedPodInfo *SchedulingQueue::Unschedulable(const std::string &key) const {
    auto it = unschedulable_.find(key);
    return it == unschedulable_.end() ? nullptr : &it->second;
}

bool SchedulingQueue::PodMatchesEvent(const framework::QueuedPodInfo &pinfo, const ClusterEvent &e) const {
    if (e.IsWildCard()) return true;  // queue.go:167-190
    for (const auto &kv : event_map_) {
        const ClusterEvent &evt = kv.first;
        const bool match = evt.IsWildCard() || (evt.resource == e.resource && (evt.action & e.action) != 0);
        if (!match) continue;
        for (const auto &name : kv.second)
            if (pinfo.UnschedulablePlugins.count(name)) return true;
    }
    return false;
}

std::chrono::nanoseconds SchedulingQueue::CalculateBackoffDuration(const framework::QueuedPodInfo &pinfo) {
    // queue.go:218-235: initial 1 s, doubled per attempt beyond the first, max 10 s
    const std::chrono::nanoseconds initial = std::chrono::seconds(1), max = std::chrono::seconds(10);
    std::chrono::nanoseconds d = initial;
    for (int i = 1; i < pinfo.attempts; ++i) {
        if (d > max - d) return max;
        d += d;
    }
    return d;
}

bool SchedulingQueue::IsPodBackingoff(const framework::QueuedPodInfo &pinfo) const {  // queue.go:206-216
    return pinfo.timestamp + CalculateBackoffDuration(pinfo) > Now();
}

void SchedulingQueue::MoveAllToActiveOrBackoffQueue(const ClusterEvent &e) {  // queue.go:54-82
    std::vector<std::string> moved;
    for (auto &kv : unschedulable_) {
        framework::QueuedPodInfo &p = kv.second;
        // an empty UnschedulablePlugins set (a non-FitError failure) moves on any event
        if (!p.UnschedulablePlugins.empty() && !PodMatchesEvent(p, e)) continue;
        if (IsPodBackingoff(p)) backoff_.push_back(p);  // never flushed (queue.go:136-139)
        else active_.push_back(p);
        moved.push_back(kv.first);
    }
    for (const auto &k : moved) unschedulable_.erase(k);
}

// ------------------------------------------------------------------ encoders
int NameDigit(const std::string &name) {
    if (name.empty()) throw std::invalid_argument("empty object name");  // the reference would panic
    const char c = name.back();
    return (c >= '0' && c <= '9') ? c - '0' : -1;
}

namespace {
constexpr int64_t kDefaultMilliCPURequest = 100;             // k8s@v1.22.0 util/non_zero.go
constexpr int64_t kDefaultMemoryRequest = 200ll * 1024 * 1024;

int64_t get(const std::optional<int64_t> &v, int64_t dflt) { return v ? *v : dflt; }
}  // namespace

ms_pod_rec EncodePod(const v1::Pod &pod, uint32_t ordinal) {
    ms_pod_rec r{};
    r.ordinal = ordinal;
    r.name_digit = (int8_t)NameDigit(pod.name);
    r.tolerates_unschedulable = v1::TolerationsTolerateTaint(
        pod.tolerations, v1::Taint{v1::kTaintNodeUnschedulable, "", v1::kTaintEffectNoSchedule});
    // Fit PreFilter (computePodResourceRequest) and calculateResource's non-zero pair
    int64_t rc = 0, rm = 0, nc = 0, nm = 0;
    for (const auto &c : pod.containers) {
        rc += get(c.requests.cpu_milli, 0);
        rm += get(c.requests.memory, 0);
        nc += get(c.requests.cpu_milli, kDefaultMilliCPURequest);
        nm += get(c.requests.memory, kDefaultMemoryRequest);
    }
    for (const auto &c : pod.init_containers) {
        rc = std::max(rc, get(c.requests.cpu_milli, 0));
        rm = std::max(rm, get(c.requests.memory, 0));
        nc = std::max(nc, get(c.requests.cpu_milli, kDefaultMilliCPURequest));
        nm = std::max(nm, get(c.requests.memory, kDefaultMemoryRequest));
    }
    if (pod.overhead) {
        rc += get(pod.overhead->cpu_milli, 0);
        rm += get(pod.overhead->memory, 0);
        nc += get(pod.overhead->cpu_milli, 0);
        nm += get(pod.overhead->memory, 0);
    }
    r.req_milli_cpu = rc;
    r.req_memory = rm;
    r.nonzero_milli_cpu = nc;
    r.nonzero_memory = nm;
    return r;
}

std::string UnsupportedRequest(const v1::Pod &pod) {
    for (const auto &c : pod.containers)
        if (!c.requests.other.empty()) return c.requests.other.begin()->first;
    for (const auto &c : pod.init_containers)
        if (!c.requests.other.empty()) return c.requests.other.begin()->first;
    if (pod.overhead && !pod.overhead->other.empty()) return pod.overhead->other.begin()->first;
    return "";
}

ms_node_rec EncodeNode(const v1::Node &node, const NodeUsage &u) {
    ms_node_rec r{};
    const int d = NameDigit(node.name);
    r.unschedulable = node.unschedulable ? 1 : 0;
    r.name_digit = d >= 0 ? (uint8_t)d : 0xFF;
    r.allowed_pods = (int32_t)get(node.allocatable.pods, 110);
    r.pod_count = u.pods;
    r.alloc_milli_cpu = get(node.allocatable.cpu_milli, 0);
    r.alloc_memory = get(node.allocatable.memory, 0);
    r.req_milli_cpu = u.req_cpu;
    r.req_memory = u.req_mem;
    r.nonzero_milli_cpu = u.nz_cpu;
    r.nonzero_memory = u.nz_mem;
    return r;
}

// ----------------------------------------------------------------- scheduler
namespace {
void register_events(const std::string &name, std::map<ClusterEvent, std::set<std::string>> &m,
                     const std::vector<ClusterEvent> &evts) {  // initialize.go:159-167
    for (const auto &e : evts) m[e].insert(name);
}
}  // namespace

Scheduler::Scheduler(const Options &opt) : opt_(opt), ordinals_(opt.max_nodes) {
    // createFilterPlugins / createScorePlugins (initialize.go:80-121); the
    // resource-aware set adds NodeResourcesFit to both extension points.
    filter_.push_back(std::make_unique<NodeUnschedulable>());
    score_.push_back(std::make_unique<NodeNumber>());
    if (opt.plugins == PluginSet::NU_NRF_NN_LA) {
        filter_.push_back(std::make_unique<NodeResourcesFit>());
        score_.push_back(std::make_unique<NodeResourcesFit>());
    }
    // eventsToRegister (initialize.go:140-157). Faithful to the reference:
    // NodeNumber's events are registered under NodeUnschedulable's name (:154).
    NodeUnschedulable nu;
    NodeNumber nn;
    register_events(nu.Name(), event_map_, nu.EventsToRegister());
    register_events(nu.Name(), event_map_, nn.EventsToRegister());
    if (opt.plugins == PluginSet::NU_NRF_NN_LA) {
        NodeResourcesFit f;
        register_events(f.Name(), event_map_, f.EventsToRegister());
    }
    for (const auto &kv : event_map_) gvk_map_[kv.first.resource] |= kv.first.action;  // unionedGVKs
    queue_ = std::make_unique<SchedulingQueue>(event_map_, opt.clock);

    ms_config cfg{};
    cfg.device = opt.device;
    cfg.plugin_set = (int32_t)opt.plugins;
    cfg.max_nodes = opt.max_nodes;
    cfg.node_base = 0;
    cfg.max_batch = 1u << 14;
    cfg.seed = opt.seed;
    const int rc = ms_create(&cfg, &ctx_);
    if (rc != MS_OK) throw std::runtime_error(std::string("ms_create: ") + ms_last_error(nullptr));
    names_.assign(opt.max_nodes, std::string());
}

Scheduler::~Scheduler() {
    if (ctx_) ms_destroy(ctx_);
}

uint32_t Scheduler::Gvk(const std::string &gvk) const {
    auto it = gvk_map_.find(gvk);
    return it == gvk_map_.end() ? 0 : it->second;
}

const NodeUsage *Scheduler::Usage(const std::string &node) const {
    auto it = usage_.find(node);
    return it == usage_.end() ? nullptr : &it->second;
}

OrdinalAllocator::OrdinalAllocator(uint32_t capacity) : cap_(capacity) {
    for (uint32_t d = 0; d < 10; ++d) next_[d] = d;
}

uint32_t OrdinalAllocator::LowestAny() {
    uint32_t best = UINT32_MAX, bd = 10;
    for (uint32_t d = 0; d < 10; ++d) {
        const uint32_t o = free_[d].empty() ? next_[d] : *free_[d].begin();
        if (o < cap_ && o < best) {
            best = o;
            bd = d;
        }
    }
    if (bd == 10) throw std::length_error("node table full");
    if (!free_[bd].empty() && *free_[bd].begin() == best) free_[bd].erase(free_[bd].begin());
    else next_[bd] += 10;
    return best;
}

bool OrdinalAllocator::Skewed() const {
    const uint32_t mx = *std::max_element(count_, count_ + 10);
    return live_ >= kSkewMinLive && 100ull * mx > (uint64_t)kSkewBreakEvenX10 * live_;
}

// (live_ and count_ already include the node being placed)
uint32_t OrdinalAllocator::Pick(int digit) {
    const bool has = digit >= 0 && digit <= 9;
    const uint64_t spread = kSpreadSlack + 2ull * live_;  // (skewed name digits)
    if (Skewed()) return LowestAny();                     // dense: cheaper than any aligned spread
    if (has && !free_[digit].empty() && *free_[digit].begin() < spread) {
        const uint32_t o = *free_[digit].begin();
        free_[digit].erase(free_[digit].begin());
        return o;
    }
    if (has && next_[digit] < cap_ && next_[digit] < spread) {
        const uint32_t o = next_[digit];
        next_[digit] += 10;
        return o;
    }
    return LowestAny();  // no digit, the digit's residue is full, or its slot is too far out
}

uint32_t OrdinalAllocator::Allocate(int digit) {
    const bool has = digit >= 0 && digit <= 9;
    if (has) ++count_[digit];
    ++live_;
    uint32_t o;
    try {
        o = Pick(digit);
    } catch (...) {  // (full: the shares stay as they were)
        --live_;
        if (has) --count_[digit];
        throw;
    }
    high_ = std::max(high_, o + 1);
    return o;
}

void OrdinalAllocator::Release(uint32_t o, int digit) {
    free_[o % 10].insert(o);
    if (live_) --live_;
    if (digit >= 0 && digit <= 9 && count_[digit]) --count_[digit];
}

uint32_t OrdinalAllocator::HighWater() const { return high_; }

uint32_t Scheduler::NodeOrdinal(const std::string &name, bool create) {
    auto it = ordinal_.find(name);
    if (it != ordinal_.end()) return it->second;
    if (!create) throw std::out_of_range("unknown node " + name);
    const uint32_t o = ordinals_.Allocate(NameDigit(name));
    ordinal_[name] = o;
    names_[o] = name;
    return o;
}

void Scheduler::OnPodAdd(const v1::Pod &pod) {  // eventhandler.go:20-35,84-90
    if (!pod.node_name.empty()) return;         // assignedPod (:80-82)
    queue_->Add(pod);
}

void Scheduler::OnNodeAdd(const v1::Node &node) {  // eventhandler.go:39-44
    const uint32_t o = NodeOrdinal(node.name, true);
    nodes_[node.name] = node;
    const ms_node_rec rec = EncodeNode(node, usage_[node.name]);
    if (ms_nodes_upsert(ctx_, 1, &o, &rec) != MS_OK) throw std::runtime_error(ms_last_error(ctx_));
    if (Gvk(framework::kNode) & framework::Add)
        queue_->MoveAllToActiveOrBackoffQueue({framework::kNode, framework::Add, "NodeAdd"});
}

void Scheduler::OnNodeUpdate(const v1::Node &, const v1::Node &node) {  // eventhandler.go:45-50
    const uint32_t o = NodeOrdinal(node.name, true);
    nodes_[node.name] = node;
    const ms_node_rec rec = EncodeNode(node, usage_[node.name]);
    if (ms_nodes_upsert(ctx_, 1, &o, &rec) != MS_OK) throw std::runtime_error(ms_last_error(ctx_));
    if (Gvk(framework::kNode) & framework::Update)
        queue_->MoveAllToActiveOrBackoffQueue({framework::kNode, framework::Update, "NodeUpdate"});
}

void Scheduler::OnNodeDelete(const v1::Node &node) {  // eventhandler.go:51-56
    auto it = ordinal_.find(node.name);
    if (it == ordinal_.end()) return;
    const uint32_t o = it->second;
    if (ms_nodes_delete(ctx_, 1, &o) != MS_OK) throw std::runtime_error(ms_last_error(ctx_));
    ordinal_.erase(it);
    names_[o].clear();
    ordinals_.Release(o, NameDigit(node.name));
    nodes_.erase(node.name);
    usage_.erase(node.name);
    if (Gvk(framework::kNode) & framework::Delete)
        queue_->MoveAllToActiveOrBackoffQueue({framework::kNode, framework::Delete, "NodeDelete"});
}

void Scheduler::ErrorFunc(const v1::Pod &pod, const framework::ScheduleError &err) {  // minisched.go:283-298
    framework::QueuedPodInfo p;  // a fresh PodInfo, as the reference builds one
    p.pod = pod;
    if (err.fit_error) p.UnschedulablePlugins = err.diagnosis.UnschedulablePlugins;
    queue_->AddUnschedulable(std::move(p));
}

ScheduleResult Scheduler::Finish(const v1::Pod &pod, const ms_pod_rec &rec, const ms_result &r) {
    ScheduleResult out;
    out.pod = pod.name;
    if (r.code == MS_CODE_UNSCHEDULABLE) {  // FitError (minisched.go:143-148)
        out.kind = ScheduleResult::Unschedulable;
        out.error.fit_error = true;
        if (r.plugin_mask & MS_MASK_NODE_UNSCHEDULABLE) out.error.diagnosis.UnschedulablePlugins.insert("NodeUnschedulable");
        if (r.plugin_mask & MS_MASK_NODE_RESOURCES_FIT) out.error.diagnosis.UnschedulablePlugins.insert("NodeResourcesFit");
        out.error.message = "0/" + std::to_string(ordinal_.size()) + " nodes are available";
        ErrorFunc(pod, out.error);
        return out;
    }
    if (r.code == MS_CODE_ERROR) {  // NodeNumber.Score error; the reference hands ErrorFunc a nil err (:73)
        out.kind = ScheduleResult::Error;
        out.error.message = "running score plugins: not found";
        ErrorFunc(pod, out.error);
        return out;
    }
    out.node = names_.at((uint32_t)r.node);
    out.score = r.score;
    // the device already assumed the pod on the node (NodeInfo.AddPod)
    NodeUsage &u = usage_[out.node];
    u.req_cpu += rec.req_milli_cpu;
    u.req_mem += rec.req_memory;
    u.nz_cpu += rec.nonzero_milli_cpu;
    u.nz_mem += rec.nonzero_memory;
    u.pods += 1;
    if (opt_.binder && !opt_.binder(pod, out.node)) {  // bind failed: forget + re-queue (:104-108)
        const uint32_t o = (uint32_t)r.node;
        ms_uncommit_bind(ctx_, o, &rec);
        u.req_cpu -= rec.req_milli_cpu;
        u.req_mem -= rec.req_memory;
        u.nz_cpu -= rec.nonzero_milli_cpu;
        u.nz_mem -= rec.nonzero_memory;
        u.pods -= 1;
        out.kind = ScheduleResult::Error;
        out.error.message = "binding rejected";
        ErrorFunc(pod, out.error);
        return out;
    }
    out.kind = ScheduleResult::Scheduled;
    return out;
}

std::vector<ScheduleResult> Scheduler::ScheduleBatch(size_t k) {
    std::vector<v1::Pod> pods;
    std::vector<ms_pod_rec> recs;
    std::vector<ScheduleResult> out;
    // pods NodeResourcesFit would check on a resource the records cannot carry:
    // a plain Error (ErrorFunc, empty plugin set), in queue order among the
    // device results; they bind nothing, so the other pods' sequential outcomes
    // are those of the queue without them
    std::vector<std::pair<size_t, ScheduleResult>> refused;
    while (pods.size() + refused.size() < k) {
        auto p = queue_->NextPod();
        if (!p) break;
        auto it = pod_ordinal_.find(p->uid.empty() ? SchedulingQueue::KeyFunc(*p) : p->uid);
        uint32_t o;
        if (it == pod_ordinal_.end()) {
            o = next_pod_ordinal_++;
            pod_ordinal_[p->uid.empty() ? SchedulingQueue::KeyFunc(*p) : p->uid] = o;
        } else {
            o = it->second;
        }
        if (opt_.plugins == PluginSet::NU_NRF_NN_LA) {
            const std::string bad = UnsupportedRequest(*p);
            if (!bad.empty()) {
                ScheduleResult r;
                r.kind = ScheduleResult::Error;
                r.pod = p->name;
                r.error.message = "NodeResourcesFit: request for " + bad +
                                  " cannot be evaluated on the device (cpu and memory only)";
                ErrorFunc(*p, r.error);
                refused.emplace_back(pods.size() + refused.size(), std::move(r));
                continue;
            }
        }
        recs.push_back(EncodePod(*p, o));
        pods.push_back(std::move(*p));
    }
    auto merge = [&refused](std::vector<ScheduleResult> dev) {  // refused pods back at their queue places
        std::vector<ScheduleResult> all;
        size_t j = 0, d = 0;
        for (size_t i = 0; i < dev.size() + refused.size(); ++i)
            all.push_back(j < refused.size() && refused[j].first == i ? refused[j++].second : dev[d++]);
        return all;
    };
    if (pods.empty()) return merge({});
    std::vector<ms_result> res(pods.size());
    const int rc = ms_schedule_batch(ctx_, (uint32_t)pods.size(), recs.data(), MS_MODE_SEQUENTIAL, res.data());
    if (rc != MS_OK) {  // device failure: every pod stays re-queueable (a plain error)
        for (const auto &p : pods) {
            ScheduleResult r;
            r.kind = ScheduleResult::Error;
            r.pod = p.name;
            r.error.message = ms_last_error(ctx_);
            ErrorFunc(p, r.error);
            out.push_back(r);
        }
        return merge(std::move(out));
    }
    for (size_t i = 0; i < pods.size(); ++i) out.push_back(Finish(pods[i], recs[i], res[i]));
    return merge(std::move(out));
}

ScheduleResult Scheduler::ScheduleOne() {
    auto v = ScheduleBatch(1);
    return v.empty() ? ScheduleResult{} : v[0];
}

}  // namespace minisched
