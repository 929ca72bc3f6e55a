// test_host.cpp — tests of the C++ host mirror (mini-kube-scheduler_amd/csrc/host).
//
//   ms_host_test cpu   queue / events / encoders / tolerations (no device)
//   ms_host_test gpu   scheduling through the device (README scenario etc.)
//
// The GPU cases replay the reference's only end-to-end scenario (sched.go:70-140)
// through the same objects and events the Go scheduler would see.
#include <stdexcept>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <set>
#include <vector>

#include "minisched.h"

using namespace minisched;
using Clock = std::chrono::steady_clock;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                                     \
    do {                                                                                \
        if (!(cond)) {                                                                  \
            std::fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);      \
            ++g_fail;                                                                   \
            return;                                                                     \
        }                                                                               \
    } while (0)

static void run(const char *name, const std::function<void()> &fn) {
    const int before = g_fail;
    fn();
    if (g_fail == before) {
        ++g_pass;
        std::printf("ok   %s\n", name);
    } else {
        std::printf("FAIL %s\n", name);
    }
}

struct FakeClock {
    Clock::time_point now = Clock::time_point(std::chrono::seconds(1000));
    SchedulingQueue::Clock fn() {
        return [this] { return now; };
    }
    void advance(double s) { now += std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(s)); }
};

static v1::Pod pod(const std::string &name, int64_t cpu = -1, int64_t mem = -1) {
    v1::Pod p;
    p.name = name;
    p.uid = "uid-" + name;
    v1::Container c;
    c.name = "container1";
    if (cpu >= 0) c.requests.cpu_milli = cpu;
    if (mem >= 0) c.requests.memory = mem;
    p.containers.push_back(c);
    return p;
}

static v1::Node node(const std::string &name, bool unsched = false, int64_t cpu = 4000, int64_t mem = 8ll << 30) {
    v1::Node n;
    n.name = name;
    n.unschedulable = unsched;
    n.allocatable.cpu_milli = cpu;
    n.allocatable.memory = mem;
    n.allocatable.pods = 110;
    return n;
}

// ---------------------------------------------------------------------- CPU
static void cpu_tests() {
    run("toleration matching (core/v1 ToleratesTaint)", [] {
        v1::Taint t{v1::kTaintNodeUnschedulable, "", v1::kTaintEffectNoSchedule};
        CHECK((v1::Toleration{v1::kTaintNodeUnschedulable, "Exists", "", "NoSchedule"}.ToleratesTaint(t)));
        CHECK((v1::Toleration{"", "Exists", "", ""}.ToleratesTaint(t)));
        CHECK((v1::Toleration{v1::kTaintNodeUnschedulable, "", "", ""}.ToleratesTaint(t)));
        CHECK(!(v1::Toleration{v1::kTaintNodeUnschedulable, "Equal", "x", ""}.ToleratesTaint(t)));
        CHECK(!(v1::Toleration{v1::kTaintNodeUnschedulable, "Exists", "", "NoExecute"}.ToleratesTaint(t)));
        CHECK(!(v1::Toleration{"other", "Exists", "", ""}.ToleratesTaint(t)));
        CHECK(!(v1::Toleration{v1::kTaintNodeUnschedulable, "Bogus", "", ""}.ToleratesTaint(t)));
    });
    run("encoders: name digits, requests, non-zero defaults", [] {
        CHECK(NameDigit("node10") == 0 && NameDigit("pod7") == 7 && NameDigit("nodeA") == -1);
        ms_pod_rec r = EncodePod(pod("pod3"), 42);
        CHECK(r.ordinal == 42 && r.name_digit == 3 && r.tolerates_unschedulable == 0);
        CHECK(r.req_milli_cpu == 0 && r.req_memory == 0);
        CHECK(r.nonzero_milli_cpu == 100 && r.nonzero_memory == 200ll * 1024 * 1024);
        v1::Pod p = pod("podZ", 0, 0);
        p.init_containers.push_back({"init", {700, 1 << 20, {}, {}}});
        p.overhead = v1::ResourceList{50, 10, {}, {}};
        r = EncodePod(p, 1);
        CHECK(r.name_digit == -1);
        CHECK(r.req_milli_cpu == 750 && r.req_memory == (1 << 20) + 10);
        CHECK(r.nonzero_milli_cpu == 750 && r.nonzero_memory == (1 << 20) + 10);
        ms_node_rec n = EncodeNode(node("nodeQ", true, 1000, 2000), NodeUsage{5, 6, 7, 8, 9});
        CHECK(n.unschedulable == 1 && n.name_digit == 0xFF && n.allowed_pods == 110);
        CHECK(n.req_milli_cpu == 5 && n.nonzero_memory == 8 && n.pod_count == 9);
    });
    run("encoders: requests the records cannot carry are named (VERDICT r5 item 3)", [] {
        CHECK(UnsupportedRequest(pod("pod1", 100, 1 << 20)).empty());
        v1::Pod g = pod("pod2");
        g.containers[0].requests.other["amd.com/gpu"] = 1;  // a GPU-only pod: no cpu / memory request
        CHECK(UnsupportedRequest(g) == "amd.com/gpu");
        v1::Pod e = pod("pod3", 100);
        e.init_containers.push_back({"init", {}});
        e.init_containers[0].requests.other["ephemeral-storage"] = 1ll << 30;
        CHECK(UnsupportedRequest(e) == "ephemeral-storage");
        v1::Pod o = pod("pod4", 100);
        o.overhead = v1::ResourceList{};
        o.overhead->other["hugepages-2Mi"] = 0;  // an explicit 0 is refused too
        CHECK(UnsupportedRequest(o) == "hugepages-2Mi");
        v1::Node n = node("node1");
        n.allocatable.other["ephemeral-storage"] = 100ll << 30;  // node side: accepted, ignored
        CHECK(EncodeNode(n, NodeUsage{}).alloc_milli_cpu == 4000);
    });
    run("ordinal allocator: ordinal % 10 == name digit, holes reused", [] {
        OrdinalAllocator a(100);
        // informer Add order with arbitrary name digits
        const int digits[] = {7, 7, 7, 3, -1, 0, 7, -1, 9, 3};
        std::vector<uint32_t> got;
        for (int d : digits) got.push_back(a.Allocate(d));
        CHECK(got[0] == 7 && got[1] == 17 && got[2] == 27 && got[3] == 3 && got[6] == 37 && got[9] == 13);
        CHECK(got[4] == 0 && got[7] == 1);  // no digit: the lowest free ordinal of any residue
        CHECK(got[5] == 10 && got[8] == 9);
        for (size_t i = 0; i < got.size(); ++i)
            if (digits[i] >= 0) CHECK((int)(got[i] % 10) == digits[i]);
        a.Release(17, 7);
        CHECK(a.Allocate(7) == 17);  // its residue's hole first
        a.Release(27, 7);
        CHECK(a.Allocate(-1) == 2);  // (2 < 27)
        // every 30 consecutive ordinals hold at most 3 of one digit
        OrdinalAllocator b(3000);
        uint64_t x = 12345;
        std::vector<int> dig(3000, -2);
        for (int i = 0; i < 2500; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            const int d = (int)((x >> 33) % 10);
            dig[b.Allocate(d)] = d;
        }
        for (uint32_t g = 0; g + 30 <= 3000; g += 30)
            for (int d = 0; d < 10; ++d) {
                int c = 0;
                for (uint32_t i = g; i < g + 30; ++i) c += dig[i] == d;
                CHECK(c <= 3);
            }
        OrdinalAllocator full(12);
        for (int i = 0; i < 12; ++i) (void)full.Allocate(5);  // residue 5 has 5 only: the rest spill
        bool threw = false;
        try {
            (void)full.Allocate(5);
        } catch (const std::length_error &) {
            threw = true;
        }
        CHECK(threw && full.HighWater() == 12);
        // skewed digits: aligned slots only within kSpreadSlack + 2 x (live + 1), then dense
        OrdinalAllocator sk(100000);
        std::set<uint32_t> seen;
        for (int i = 0; i < 5000; ++i) seen.insert(sk.Allocate(0));
        CHECK(seen.size() == 5000 && sk.HighWater() <= 2 * 5000 + OrdinalAllocator::kSpreadSlack + 2);
        // skew fallback: dense once 100 x max count > 26 x live, live >= 100
        CHECK(sk.Skewed() && sk.HighWater() <= 5000 + OrdinalAllocator::kSpreadSlack);
        OrdinalAllocator t(10000);
        for (int i = 0; i < 100; ++i) (void)t.Allocate(i < 26 ? 0 : 1 + i % 9);
        CHECK(!t.Skewed());  // 26 % of one digit
        (void)t.Allocate(0);
        CHECK(t.Skewed());   // 27 of 101
        // 70 % zeros: the table stays ~n rows
        OrdinalAllocator s70(100000);
        std::vector<std::pair<uint32_t, int>> held;
        uint64_t y = 777;
        for (int i = 0; i < 20000; ++i) {
            y = y * 6364136223846793005ull + 1442695040888963407ull;
            const int d = ((y >> 33) % 100) < 70 ? 0 : (int)((y >> 40) % 10);
            held.push_back({s70.Allocate(d), d});
        }
        CHECK(s70.Skewed() && s70.HighWater() <= 20000 + OrdinalAllocator::kSpreadSlack);
        for (const auto &h : held)
            if (h.second == 0) s70.Release(h.first, 0);
        CHECK(!s70.Skewed() && s70.Allocate(3) % 10 == 3);  // alignment back
    });
    run("queue: FIFO, backoff 1 s, event matching (queue.go)", [] {
        FakeClock clk;
        std::map<framework::ClusterEvent, std::set<std::string>> m;
        m[{framework::kNode, framework::Add | framework::UpdateNodeTaint, ""}].insert("NodeUnschedulable");
        SchedulingQueue q(m, clk.fn());
        q.Add(pod("pod1"));
        q.Add(pod("pod2"));
        CHECK(q.NextPod()->name == "pod1");
        framework::QueuedPodInfo a;
        a.pod = pod("pod1");
        a.UnschedulablePlugins = {"NodeUnschedulable"};
        q.AddUnschedulable(a);
        framework::QueuedPodInfo b;
        b.pod = pod("pod9");
        b.UnschedulablePlugins = {"NodeResourcesFit"};
        q.AddUnschedulable(b);
        framework::QueuedPodInfo c;  // plain error: empty plugin set moves on any event
        c.pod = pod("podX");
        q.AddUnschedulable(c);
        CHECK(q.UnschedulableLen() == 3);
        // an event no plugin registered: only the plain-error pod moves (into backoffQ: < 1 s)
        q.MoveAllToActiveOrBackoffQueue({framework::kPod, framework::Delete, "PodDelete"});
        CHECK(q.UnschedulableLen() == 2 && q.BackoffLen() == 1);
        clk.advance(3.0);  // sched.go waits 3 s before adding node10
        q.MoveAllToActiveOrBackoffQueue({framework::kNode, framework::Add, "NodeAdd"});
        CHECK(q.UnschedulableLen() == 1 && q.Unschedulable("pod9_default") != nullptr);
        CHECK(q.ActiveLen() == 2);  // pod2 + pod1
        CHECK(q.NextPod()->name == "pod2" && q.NextPod()->name == "pod1");
        CHECK(!q.NextPod().has_value());
        // within the backoff window a matching pod goes to backoffQ, which is never flushed
        framework::QueuedPodInfo d;
        d.pod = pod("pod4");
        d.UnschedulablePlugins = {"NodeUnschedulable"};
        q.AddUnschedulable(d);
        clk.advance(0.5);
        q.MoveAllToActiveOrBackoffQueue({framework::kNode, framework::UpdateNodeTaint, "NodeUpdate"});
        CHECK(q.BackoffLen() == 2 && q.ActiveLen() == 0);
    });
    run("backoff duration (queue.go:218-235)", [] {
        framework::QueuedPodInfo p;
        using std::chrono::seconds;
        p.attempts = 0;
        CHECK(SchedulingQueue::CalculateBackoffDuration(p) == seconds(1));
        p.attempts = 3;
        CHECK(SchedulingQueue::CalculateBackoffDuration(p) == seconds(4));
        p.attempts = 10;
        CHECK(SchedulingQueue::CalculateBackoffDuration(p) == seconds(10));
    });
}

// ---------------------------------------------------------------------- GPU
static void gpu_tests() {
    run("plugin wiring and events (initialize.go)", [] {
        Scheduler s(Scheduler::Options{});
        CHECK(s.FilterPlugins().size() == 1 && s.FilterPlugins()[0]->Name() == "NodeUnschedulable");
        CHECK(s.ScorePlugins().size() == 1 && s.ScorePlugins()[0]->Name() == "NodeNumber");
        // NodeNumber's Node/Add lands under NodeUnschedulable's name (initialize.go:154)
        framework::ClusterEvent nn{framework::kNode, framework::Add, ""};
        CHECK(s.EventMap().count(nn) && s.EventMap().at(nn).count("NodeUnschedulable"));
        CHECK((s.Gvk(framework::kNode) & framework::Add) && (s.Gvk(framework::kNode) & framework::UpdateNodeTaint));
        CHECK(!(s.Gvk(framework::kNode) & framework::Delete));
    });
    run("README scenario end to end (sched.go:70-140)", [] {
        FakeClock clk;
        Scheduler::Options o;
        o.clock = clk.fn();
        std::vector<std::pair<std::string, std::string>> bound;
        o.binder = [&](const v1::Pod &p, const std::string &n) {
            bound.push_back({p.name, n});
            return true;
        };
        Scheduler s(o);
        for (int i = 0; i < 9; ++i) s.OnNodeAdd(node("node" + std::to_string(i), true));  // :74-85
        s.OnPodAdd(pod("pod1"));                                                           // :91-101
        ScheduleResult r = s.ScheduleOne();
        CHECK(r.kind == ScheduleResult::Unschedulable);
        CHECK(r.error.fit_error && r.error.diagnosis.UnschedulablePlugins == std::set<std::string>{"NodeUnschedulable"});
        CHECK(s.Queue().UnschedulableLen() == 1 && bound.empty());  // :109-119 "not bound yet"
        CHECK(s.ScheduleOne().kind == ScheduleResult::NoPod);
        clk.advance(3.0);
        s.OnNodeAdd(node("node10"));  // :121-129 -> NodeAdd event re-activates pod1
        CHECK(s.Queue().ActiveLen() == 1);
        r = s.ScheduleOne();
        CHECK(r.kind == ScheduleResult::Scheduled && r.node == "node10" && r.score == 0);
        CHECK(bound.size() == 1 && bound[0].second == "node10");
        CHECK(s.Usage("node10")->pods == 1);
    });
    run("NodeNumber scoring and non-digit pod error", [] {
        Scheduler s(Scheduler::Options{});
        s.OnNodeAdd(node("node17"));
        s.OnNodeAdd(node("nodeA"));
        s.OnNodeAdd(node("node8"));
        s.OnPodAdd(pod("pod7"));
        ScheduleResult r = s.ScheduleOne();
        CHECK(r.kind == ScheduleResult::Scheduled && r.node == "node17" && r.score == 10);
        s.OnPodAdd(pod("podX"));
        r = s.ScheduleOne();
        CHECK(r.kind == ScheduleResult::Error && !r.error.fit_error);
        CHECK(s.Queue().UnschedulableLen() == 1);
    });
    run("batch == one-by-one (sequential, resource-aware)", [] {
        auto make = [] {
            Scheduler::Options o;
            o.plugins = Scheduler::PluginSet::NU_NRF_NN_LA;
            o.seed = 7;
            auto s = std::make_unique<Scheduler>(o);
            for (int i = 0; i < 40; ++i)
                s->OnNodeAdd(node("node" + std::to_string(i), i % 7 == 0, 1000 * (1 + i % 4), (2ll << 30) * (1 + i % 3)));
            for (int j = 0; j < 300; ++j) s->OnPodAdd(pod("pod" + std::to_string(j), 100 * (1 + j % 9), (64ll << 20) * (1 + j % 5)));
            return s;
        };
        auto a = make();
        auto b = make();
        std::vector<ScheduleResult> one, batch = b->ScheduleBatch(300);
        for (int j = 0; j < 300; ++j) one.push_back(a->ScheduleOne());
        CHECK(batch.size() == 300);
        int fit = 0;
        for (int j = 0; j < 300; ++j) {
            CHECK(one[j].kind == batch[j].kind && one[j].node == batch[j].node && one[j].score == batch[j].score);
            CHECK(one[j].error.diagnosis.UnschedulablePlugins == batch[j].error.diagnosis.UnschedulablePlugins);
            fit += one[j].kind == ScheduleResult::Unschedulable;
        }
        CHECK(fit > 0);  // the cluster saturates: FitError{NodeResourcesFit...}
        for (int i = 0; i < 40; ++i) {
            const std::string n = "node" + std::to_string(i);
            const NodeUsage *ua = a->Usage(n), *ub = b->Usage(n);
            CHECK(ua && ub && ua->pods == ub->pods && ua->req_cpu == ub->req_cpu);
        }
    });
    run("unsupported requests: Error + ErrorFunc, the rest as without them (resource-aware)", [] {
        Scheduler::Options o;
        o.plugins = Scheduler::PluginSet::NU_NRF_NN_LA;
        o.seed = 5;
        auto make = [&o]() {
            auto s = std::make_unique<Scheduler>(o);
            for (int i = 0; i < 12; ++i) s->OnNodeAdd(node("node" + std::to_string(i), false, 1000, 2ll << 30));
            for (int j = 0; j < 60; ++j) {
                v1::Pod p = pod("pod" + std::to_string(j), 300, 64ll << 20);
                if (j % 7 == 3) p.containers[0].requests.other[j % 2 ? "amd.com/gpu" : "ephemeral-storage"] = 1;
                s->OnPodAdd(p);
            }
            return s;
        };
        auto a = make();
        std::vector<ScheduleResult> ra = a->ScheduleBatch(60);
        CHECK(ra.size() == 60);
        int refused = 0;
        for (int j = 0; j < 60; ++j) {
            CHECK(ra[j].pod == "pod" + std::to_string(j));
            if (j % 7 == 3) {
                CHECK(ra[j].kind == ScheduleResult::Error && !ra[j].error.fit_error && ra[j].node.empty());
                ++refused;
            }
        }
        CHECK(a->Queue().UnschedulableLen() >= (size_t)refused);
        // every refused pod is parked with an empty plugin set (moves on any event)
        CHECK(a->Queue().Unschedulable("pod3_default") && a->Queue().Unschedulable("pod3_default")->UnschedulablePlugins.empty());
        // usage on the device equals the host's books (refused pods bound nothing)
        int64_t req = 0;
        int pods = 0;
        for (int i = 0; i < 12; ++i) {
            const NodeUsage *u = a->Usage("node" + std::to_string(i));
            if (u) { req += u->req_cpu; pods += u->pods; }
        }
        int sched = 0;
        for (const auto &r : ra) sched += r.kind == ScheduleResult::Scheduled;
        CHECK(pods == sched && req == 300ll * sched);
    });
    run("node delete and update (device deltas)", [] {
        FakeClock clk;
        Scheduler::Options o;
        o.clock = clk.fn();
        Scheduler s(o);
        s.OnNodeAdd(node("node1"));
        s.OnNodeAdd(node("node2"));
        s.OnNodeDelete(node("node1"));
        s.OnPodAdd(pod("pod1"));
        ScheduleResult r = s.ScheduleOne();
        CHECK(r.kind == ScheduleResult::Scheduled && r.node == "node2");  // node1 gone
        s.OnNodeUpdate(node("node2"), node("node2", true));                // cordoned
        s.OnPodAdd(pod("pod2"));
        r = s.ScheduleOne();
        CHECK(r.kind == ScheduleResult::Unschedulable);
        clk.advance(2.0);
        s.OnNodeUpdate(node("node2", true), node("node2"));  // uncordoned: UpdateNodeTaint-compatible event
        r = s.ScheduleOne();
        CHECK(r.kind == ScheduleResult::Scheduled && r.node == "node2" && s.Usage("node2")->pods == 2);
    });
    run("binder failure forgets the assumed pod", [] {
        Scheduler::Options o;
        o.plugins = Scheduler::PluginSet::NU_NRF_NN_LA;
        o.binder = [](const v1::Pod &, const std::string &) { return false; };
        Scheduler s(o);
        s.OnNodeAdd(node("node1"));
        s.OnPodAdd(pod("pod1", 500));
        ScheduleResult r = s.ScheduleOne();
        CHECK(r.kind == ScheduleResult::Error && s.Usage("node1")->pods == 0);
        ms_node_rec rec{};
        CHECK(ms_nodes_read(s.Ctx(), 0, 1, &rec) == MS_OK && rec.pod_count == 0 && rec.req_milli_cpu == 0);
    });
}

// ------------------------------------------------------------- GPU replay
// ms_host_test replay <cluster.txt> <out.txt> <seed> <plugin_set>: feeds a
// cluster through the informer handlers (OnNodeAdd in file order, then
// OnPodAdd), runs ScheduleOne until the queue is empty and writes one line per
// cycle: "pod kind node score mask" (mask: bit0 NodeUnschedulable, bit1
// NodeResourcesFit). tests/test_host_cpp.py compares that with the CPU oracle
// on the same inputs: the host mirror's queue order, ordinals, encoders and
// ErrorFunc against an independent restatement, not against itself.
//   N <name> <unschedulable 0/1> <cpu milli> <memory bytes> <pods>
//   P <name> <cpu milli or -1> <memory bytes or -1> <tolerates 0/1> <extra>
// where <extra> is "-" or "<resource name>=<quantity>" (a request the records
// cannot carry: under NodeResourcesFit that pod's cycle is a plain Error).
static int replay(const char *in_path, const char *out_path, uint64_t seed, int plugin_set) {
    FILE *f = std::fopen(in_path, "r");
    if (!f) return 2;
    Scheduler::Options o;
    o.seed = seed;
    o.plugins = plugin_set ? Scheduler::PluginSet::NU_NRF_NN_LA : Scheduler::PluginSet::NU_NN;
    o.binder = [](const v1::Pod &, const std::string &) { return true; };
    std::vector<v1::Node> nodes;
    std::vector<v1::Pod> pods;
    char kind[4], name[128];
    while (std::fscanf(f, "%3s %127s", kind, name) == 2) {
        if (kind[0] == 'N') {
            int uns;
            long long cpu, mem, np;
            if (std::fscanf(f, "%d %lld %lld %lld", &uns, &cpu, &mem, &np) != 4) return 3;
            v1::Node n = node(name, uns != 0, cpu, mem);
            n.allocatable.pods = np;
            nodes.push_back(n);
        } else {
            long long cpu, mem;
            int tol;
            char extra[128];
            if (std::fscanf(f, "%lld %lld %d %127s", &cpu, &mem, &tol, extra) != 4) return 3;
            v1::Pod p = pod(name, cpu, mem);
            if (tol) p.tolerations.push_back({v1::kTaintNodeUnschedulable, "Exists", "", ""});
            if (std::strcmp(extra, "-") != 0) {
                const char *eq = std::strchr(extra, '=');
                if (!eq) return 3;
                p.containers[0].requests.other[std::string(extra, (size_t)(eq - extra))] = std::atoll(eq + 1);
            }
            pods.push_back(p);
        }
    }
    std::fclose(f);
    o.max_nodes = (uint32_t)std::max<size_t>(1, nodes.size());
    Scheduler s(o);
    for (const auto &n : nodes) s.OnNodeAdd(n);
    for (const auto &p : pods) s.OnPodAdd(p);
    FILE *out = std::fopen(out_path, "w");
    if (!out) return 2;
    for (;;) {
        const ScheduleResult r = s.ScheduleOne();
        if (r.kind == ScheduleResult::NoPod) break;
        unsigned mask = 0;
        for (const auto &pl : r.error.diagnosis.UnschedulablePlugins)
            mask |= pl == "NodeUnschedulable" ? 1u : pl == "NodeResourcesFit" ? 2u : 0u;
        std::fprintf(out, "%s %d %s %lld %u\n", r.pod.c_str(), (int)r.kind, r.node.empty() ? "-" : r.node.c_str(),
                     (long long)r.score, mask);
    }
    std::fclose(out);
    std::printf("replayed %zu pods on %zu nodes\n", pods.size(), nodes.size());
    return 0;
}

int main(int argc, char **argv) {
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    if (mode == "replay" && argc == 6) return replay(argv[2], argv[3], std::strtoull(argv[4], nullptr, 10), std::atoi(argv[5]));
    if (mode == "cpu" || mode == "all") cpu_tests();
    if (mode == "gpu" || mode == "all") gpu_tests();
    std::printf("%d passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
