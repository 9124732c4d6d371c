// core.cpp -- C++ host mirror of the reference's Go `core` API over the C-ABI (see core.hpp).
#include "core.hpp"
#include "gosort.hpp"

#include <algorithm>
#include <cmath>
#include <fstream>
#include <numeric>
#include <sstream>
#include <thread>

namespace core {

namespace {

[[noreturn]] void panic_rs(const rs_ctx* ctx, const char* what) {
    throw Panic(std::string(what) + ": " + rs_last_error(ctx));
}

std::vector<double> flatten(const std::vector<std::vector<double>>& m, int k) {
    std::vector<double> f(m.size() * static_cast<size_t>(k));
    for (size_t r = 0; r < m.size(); ++r) std::copy(m[r].begin(), m[r].end(), f.begin() + r * k);
    return f;
}

std::vector<std::vector<double>> unflatten(const std::vector<double>& f, size_t rows, int k) {
    std::vector<std::vector<double>> m(rows);
    for (size_t r = 0; r < rows; ++r) m[r].assign(f.begin() + r * k, f.begin() + (r + 1) * k);
    return m;
}

double dot(const std::vector<double>& a, const std::vector<double>& b) {  // gonum floats.Dot
    double s = 0.0;
    for (size_t f = 0; f < a.size(); ++f) s += a[f] * b[f];
    return s;
}

int sgd_mode(const Parameters& p) {
    const std::string m = p.GetString("mode", "fast");
    if (m == "fast") return RS_SGD_FAST;
    if (m == "ordered") return RS_SGD_ORDERED;
    throw Panic("unknown mode " + m);
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// data.go

DataSet DataSet::SubSet(const std::vector<int64_t>& indices) const {
    DataSet d;
    d.Ratings.reserve(indices.size());
    d.Users.reserve(indices.size());
    d.Items.reserve(indices.size());
    for (int64_t i : indices) {
        d.Users.push_back(Users[i]);
        d.Items.push_back(Items[i]);
        d.Ratings.push_back(Ratings[i]);
    }
    return d;
}

void DataSet::KFold(int k, const std::vector<int64_t>& perm, std::vector<TrainSet>& trains,
                    std::vector<DataSet>& tests) const {
    const int64_t n = Length(), fold = n / k;
    trains.clear();
    tests.clear();
    int64_t begin = 0, end = 0;
    for (int i = 0; i < k; ++i) {  // data.go:56-68
        end += fold;
        if (i < n % k) end++;
        std::vector<int64_t> test(perm.begin() + begin, perm.begin() + end);
        std::vector<int64_t> train(perm.begin(), perm.begin() + begin);
        train.insert(train.end(), perm.begin() + end, perm.end());
        tests.push_back(SubSet(test));
        trains.push_back(NewTrainSet(SubSet(train)));
        begin = end;
    }
}

TrainSet NewTrainSet(const DataSet& raw) {
    TrainSet set;
    static_cast<DataSet&>(set) = raw;
    set.GlobalMean = raw.Length() ? std::accumulate(raw.Ratings.begin(), raw.Ratings.end(), 0.0) /
                                        static_cast<double>(raw.Length())
                                  : std::nan("");  // stat.Mean of an empty slice is NaN
    set.innerUsers.resize(raw.Length());
    set.innerItems.resize(raw.Length());
    for (int64_t t = 0; t < raw.Length(); ++t) {  // data.go:137-143
        auto it = set.InnerUserIDs.find(raw.Users[t]);
        if (it == set.InnerUserIDs.end()) it = set.InnerUserIDs.emplace(raw.Users[t], set.UserCount++).first;
        set.innerUsers[t] = it->second;
    }
    for (int64_t t = 0; t < raw.Length(); ++t) {  // data.go:145-151
        auto it = set.InnerItemIDs.find(raw.Items[t]);
        if (it == set.InnerItemIDs.end()) it = set.InnerItemIDs.emplace(raw.Items[t], set.ItemCount++).first;
        set.innerItems[t] = it->second;
    }
    return set;
}

int TrainSet::ConvertUserID(int64_t userID) const {
    auto it = InnerUserIDs.find(userID);
    return it == InnerUserIDs.end() ? newID : it->second;
}

int TrainSet::ConvertItemID(int64_t itemID) const {
    auto it = InnerItemIDs.find(itemID);
    return it == InnerItemIDs.end() ? newID : it->second;
}

const std::vector<std::vector<IDRating>>& TrainSet::UserRatings() const {
    if (userRatings.empty() && UserCount > 0) {
        userRatings.assign(UserCount, {});
        for (int64_t t = 0; t < Length(); ++t) userRatings[innerUsers[t]].push_back({innerItems[t], Ratings[t]});
    }
    return userRatings;
}

const std::vector<std::vector<IDRating>>& TrainSet::ItemRatings() const {
    if (itemRatings.empty() && ItemCount > 0) {
        itemRatings.assign(ItemCount, {});
        for (int64_t t = 0; t < Length(); ++t) itemRatings[innerItems[t]].push_back({innerUsers[t], Ratings[t]});
    }
    return itemRatings;
}

rs_ratings TrainSet::ratings_view(std::vector<double>&) const {
    rs_ratings r;
    r.nnz = Length();
    r.n_users = UserCount;
    r.n_items = ItemCount;
    r.users = innerUsers.data();
    r.items = innerItems.data();
    r.ratings = Ratings.data();
    return r;
}

DataSet LoadDataFromFile(const std::string& path, const std::string& sep) {
    std::ifstream f(path);
    if (!f) throw Panic("open " + path + ": no such file");  // data.go:293-295 log.Fatal
    DataSet d;
    std::string line;
    while (std::getline(f, line)) {
        if (line.empty()) continue;
        std::vector<std::string> fields;
        size_t pos = 0, next;
        while ((next = line.find(sep, pos)) != std::string::npos) {
            fields.push_back(line.substr(pos, next - pos));
            pos = next + sep.size();
        }
        fields.push_back(line.substr(pos));
        if (fields.size() < 3) continue;
        // data.go:302-304 parse with strconv.Atoi, which turns "3.5" and every ML-20M rating into 0
        // (Q10); this loader parses the rating as a float (documented deviation).
        d.Users.push_back(std::strtoll(fields[0].c_str(), nullptr, 10));
        d.Items.push_back(std::strtoll(fields[1].c_str(), nullptr, 10));
        d.Ratings.push_back(std::strtod(fields[2].c_str(), nullptr));
    }
    return d;
}

// ---------------------------------------------------------------------------------------------
// Estimator plumbing

rs_ctx* Estimator::context() {
    if (!ctx_) {
        rs_ctx* c = nullptr;
        if (rs_open(Params.GetInt("device", 0), &c) != RS_OK) panic_rs(nullptr, "rs_open");
        ctx_ = std::shared_ptr<rs_ctx>(c, rs_close);
    }
    return ctx_.get();
}

std::mt19937_64& Estimator::rng() {
    if (!rng_) {
        auto it = Params.find("seed");
        const uint64_t seed = it != Params.end() ? static_cast<uint64_t>(Params.GetInt("seed", 0))
                                                 : std::random_device{}();  // math/rand: unseeded (Q4)
        rng_ = std::make_unique<std::mt19937_64>(seed);
    }
    return *rng_;
}

std::vector<double> Estimator::normal_vector(int n, double mean, double std) {
    std::normal_distribution<double> d(0.0, 1.0);
    std::vector<double> v(n);
    for (auto& x : v) x = d(rng()) * std + mean;  // utils.go:74
    return v;
}

std::vector<double> Estimator::uniform_vector(int n, double low, double high) {
    std::uniform_real_distribution<double> d(0.0, 1.0);
    std::vector<double> v(n);
    for (auto& x : v) x = d(rng()) * (high - low) + low;  // utils.go:83
    return v;
}

// ---------------------------------------------------------------------------------------------
// SVD (svd.go:18-132)

std::unique_ptr<SVD> NewSVD(const Parameters& params) {
    auto s = std::make_unique<SVD>();
    s->Params = params;
    return s;
}

double SVD::Predict(int64_t userID, int64_t itemID) {
    const int u = Data.ConvertUserID(userID), i = Data.ConvertItemID(itemID);
    double ret = GlobalBias;
    if (u != newID) ret += UserBias[u];
    if (i != newID) ret += ItemBias[i];
    if (u != newID && i != newID) ret += dot(UserFactor[u], ItemFactor[i]);
    return ret;
}

void SVD::Fit(const TrainSet& trainSet) {
    const int k = Params.GetInt("nFactors", 100);
    const int epochs = Params.GetInt("nEpochs", 20);
    const double lr = Params.GetFloat64("lr", 0.005), reg = Params.GetFloat64("reg", 0.02);
    const double mean = Params.GetFloat64("initMean", 0), std = Params.GetFloat64("initStdDev", 0.1);
    Data = trainSet;
    UserFactor.assign(Data.UserCount, {});
    ItemFactor.assign(Data.ItemCount, {});
    for (auto& row : UserFactor) row = normal_vector(k, mean, std);  // svd.go:80-85: users first
    for (auto& row : ItemFactor) row = normal_vector(k, mean, std);
    UserBias.assign(Data.UserCount, 0.0);
    ItemBias.assign(Data.ItemCount, 0.0);
    GlobalBias = 0.0;
    std::vector<double> P = flatten(UserFactor, k), Q = flatten(ItemFactor, k), scratch;
    rs_ratings r = Data.ratings_view(scratch);
    rs_sgd_params p{k, epochs, lr, reg, sgd_mode(Params), RS_SGD_WB_TILE};
    if (rs_svd_fit(context(), &r, &p, P.data(), Q.data(), UserBias.data(), ItemBias.data(), &GlobalBias) != RS_OK)
        panic_rs(context(), "SVD.Fit");
    UserFactor = unflatten(P, Data.UserCount, k);
    ItemFactor = unflatten(Q, Data.ItemCount, k);
}

// ---------------------------------------------------------------------------------------------
// SVD++ (svd.go:259-433)

std::unique_ptr<SVDPP> NewSVDpp(const Parameters& params) {
    auto s = std::make_unique<SVDPP>();
    s->Params = params;
    return s;
}

double SVDPP::Predict(int64_t userID, int64_t itemID) {  // svd.go:284-314
    const int u = Data.ConvertUserID(userID), i = Data.ConvertItemID(itemID);
    double ret = GlobalBias;
    if (u != newID) ret += UserBias[u];
    if (i != newID) ret += ItemBias[i];
    if (u != newID && i != newID) {
        const size_t k = ItemFactor[i].size();
        std::vector<double> e(k, 0.0);  // svd.go:271-282
        for (const IDRating& ir : UserRatings[u])
            for (size_t f = 0; f < k; ++f) e[f] = e[f] + ImplFactor[ir.ID][f];
        const double s = std::sqrt(static_cast<double>(UserRatings[u].size()));
        for (auto& x : e) x /= s;
        double d = 0.0;
        for (size_t f = 0; f < k; ++f) d += ((0.0 + UserFactor[u][f]) + e[f]) * ItemFactor[i][f];
        ret += d;
    }
    return ret;
}

void SVDPP::Fit(const TrainSet& trainSet) {
    const int k = Params.GetInt("nFactors", 20);
    const int epochs = Params.GetInt("nEpochs", 20);
    const double lr = Params.GetFloat64("lr", 0.007), reg = Params.GetFloat64("reg", 0.02);
    const double mean = Params.GetFloat64("initMean", 0), std = Params.GetFloat64("initStdDev", 0.1);
    Data = trainSet;
    UserBias.assign(Data.UserCount, 0.0);
    ItemBias.assign(Data.ItemCount, 0.0);
    UserFactor.assign(Data.UserCount, {});
    ItemFactor.assign(Data.ItemCount, {});
    ImplFactor.assign(Data.ItemCount, {});
    for (auto& row : UserFactor) row = normal_vector(k, mean, std);  // svd.go:334-336
    for (int i = 0; i < Data.ItemCount; ++i) {                      // svd.go:337-340 interleaved
        ItemFactor[i] = normal_vector(k, mean, std);
        ImplFactor[i] = normal_vector(k, mean, std);
    }
    UserRatings = Data.UserRatings();
    GlobalBias = 0.0;
    std::vector<double> P = flatten(UserFactor, k), Q = flatten(ItemFactor, k), Y = flatten(ImplFactor, k), s;
    rs_ratings r = Data.ratings_view(s);
    rs_sgd_params p{k, epochs, lr, reg, sgd_mode(Params), RS_SGD_WB_TILE};
    if (rs_svdpp_fit(context(), &r, &p, P.data(), Q.data(), Y.data(), UserBias.data(), ItemBias.data(),
                     &GlobalBias) != RS_OK)
        panic_rs(context(), "SVDPP.Fit");
    UserFactor = unflatten(P, Data.UserCount, k);
    ItemFactor = unflatten(Q, Data.ItemCount, k);
    ImplFactor = unflatten(Y, Data.ItemCount, k);
}

// ---------------------------------------------------------------------------------------------
// NMF (svd.go:134-257)

std::unique_ptr<NMF> NewNMF(const Parameters& params) {
    auto s = std::make_unique<NMF>();
    s->Params = params;
    return s;
}

double NMF::Predict(int64_t userID, int64_t itemID) {
    const int u = Data.ConvertUserID(userID), i = Data.ConvertItemID(itemID);
    if (u != newID && i != newID) return dot(userFactor[u], itemFactor[i]);
    return 0.0;
}

void NMF::Fit(const TrainSet& trainSet) {
    const int k = Params.GetInt("nFactors", 15);
    const int epochs = Params.GetInt("nEpochs", 50);
    const double low = Params.GetFloat64("initLow", 0), high = Params.GetFloat64("initHigh", 1);
    const double reg = Params.GetFloat64("reg", 0.06);
    const bool as_written = Params.GetBool("asWritten", true);
    Data = trainSet;
    userFactor.assign(Data.UserCount, {});
    itemFactor.assign(Data.ItemCount, {});
    for (auto& row : userFactor) row = uniform_vector(k, low, high);  // svd.go:167-168
    for (auto& row : itemFactor) row = uniform_vector(k, low, high);
    std::vector<double> P = flatten(userFactor, k), Q = flatten(itemFactor, k), s;
    rs_ratings r = Data.ratings_view(s);
    if (rs_nmf_fit(context(), &r, k, epochs, reg, as_written ? 1 : 0, P.data(), Q.data()) != RS_OK)
        panic_rs(context(), "NMF.Fit");
    userFactor = unflatten(P, Data.UserCount, k);
    itemFactor = unflatten(Q, Data.ItemCount, k);
}

// ---------------------------------------------------------------------------------------------
// KNN (knn.go)

static std::unique_ptr<KNN> new_knn(const Parameters& params, const char* type) {
    auto k = std::make_unique<KNN>(type);  // knn.go:50-73: the type ignores Params (Q9)
    k->Params = params;
    return k;
}
std::unique_ptr<KNN> NewKNN(const Parameters& p) { return new_knn(p, "basic"); }
std::unique_ptr<KNN> NewKNNWithMean(const Parameters& p) { return new_knn(p, "centered"); }
std::unique_ptr<KNN> NewKNNWithZScore(const Parameters& p) { return new_knn(p, "zscore"); }
std::unique_ptr<KNN> NewKNNBaseLine(const Parameters& p) { return new_knn(p, "baseline"); }

void KNN::Fit(const TrainSet& trainSet) {  // knn.go:143-217
    const Sim sim = Params.GetSim("sim", Sim::MSD);
    const bool userBased = Params.GetBool("userBased", true);
    Data = trainSet;
    GlobalMean = trainSet.GlobalMean;
    LeftRatings = userBased ? Data.UserRatings() : Data.ItemRatings();
    RightRatings = userBased ? Data.ItemRatings() : Data.UserRatings();
    L = static_cast<int>(LeftRatings.size());
    const int R = static_cast<int>(RightRatings.size());
    if (KNNType == "centered" || KNNType == "zscore") {  // knn.go:164-166, data.go:222-235
        Means.assign(L, 0.0);
        for (int i = 0; i < L; ++i) {
            double sum = 0.0, count = 0.0;
            for (const IDRating& ir : LeftRatings[i]) {
                sum += ir.Rating;
                count++;
            }
            Means[i] = sum / count;
        }
    }
    if (KNNType == "zscore") {  // knn.go:167-177
        StdDevs.assign(L, 0.0);
        for (int i = 0; i < L; ++i) {
            double sum = 0.0, count = 0.0;
            for (const IDRating& ir : LeftRatings[i]) {
                sum += (ir.Rating - Means[i]) * (ir.Rating - Means[i]);
                count++;
            }
            StdDevs[i] = std::sqrt(sum / count) + 1e-5;
        }
    }
    if (KNNType == "baseline") {  // knn.go:179-187 -> base.go:135-163 with the KNN's Params
        std::vector<double> bu(Data.UserCount, 0.0), bi(Data.ItemCount, 0.0), s;
        double gb = 0.0;
        rs_ratings r = Data.ratings_view(s);
        if (rs_baseline_fit(context(), &r, Params.GetInt("nEpochs", 20), Params.GetFloat64("lr", 0.005),
                            Params.GetFloat64("reg", 0.02), bu.data(), bi.data(), &gb) != RS_OK)
            panic_rs(context(), "BaseLine.Fit");
        Bias = userBased ? bu : bi;
    }
    std::vector<int64_t> rowptr(L + 1, 0);
    std::vector<int32_t> ids;
    std::vector<double> vals;
    for (int i = 0; i < L; ++i) {
        rowptr[i + 1] = rowptr[i] + static_cast<int64_t>(LeftRatings[i].size());
        for (const IDRating& ir : LeftRatings[i]) {
            ids.push_back(ir.ID);
            vals.push_back(ir.Rating);
        }
    }
    Sims.assign(static_cast<size_t>(L) * L, 0.0);
    if (L > 0 && rs_knn_sims(context(), static_cast<int32_t>(sim), L, R, rowptr.data(), ids.data(),
                             vals.data(), Sims.data()) != RS_OK)
        panic_rs(context(), "KNN.Fit");
}

double KNN::Predict(int64_t userID, int64_t itemID) {  // knn.go:75-141
    const int u = Data.ConvertUserID(userID), i = Data.ConvertItemID(itemID);
    const bool userBased = Params.GetBool("userBased", true);
    const int k = Params.GetInt("k", 40), minK = Params.GetInt("mink", 1);
    const int left = userBased ? u : i, right = userBased ? i : u;
    if (left == newID || right == newID) return GlobalMean;
    const double* srow = Sims.data() + static_cast<size_t>(left) * L;
    std::vector<IDRating> cand;
    for (const IDRating& ir : RightRatings[right])
        if (!std::isnan(srow[ir.ID])) cand.push_back(ir);
    if (static_cast<int>(cand.size()) <= minK) return GlobalMean;
    // knn.go:107-108 sort.Sort: Go's pdqsort, restated call for call (gosort.hpp), so ties among equal
    // similarities end in the reference's order
    gosort::sort(static_cast<int64_t>(cand.size()),
                 [&](int64_t a, int64_t b) { return srow[cand[a].ID] > srow[cand[b].ID]; },
                 [&](int64_t a, int64_t b) { std::swap(cand[a], cand[b]); });
    const size_t nn = std::min<size_t>(k, cand.size());
    double weightSum = 0.0, weightRating = 0.0;
    for (size_t t = 0; t < nn; ++t) {
        const IDRating& o = cand[t];
        weightSum += srow[o.ID];
        double rating = o.Rating;
        if (KNNType == "centered") rating -= Means[o.ID];
        else if (KNNType == "zscore") rating = (rating - Means[o.ID]) / StdDevs[o.ID];
        else if (KNNType == "baseline") rating -= Bias[o.ID];
        weightRating += srow[o.ID] * rating;
    }
    double prediction = weightRating / weightSum;
    if (KNNType == "centered") prediction += Means[left];
    else if (KNNType == "baseline") prediction += Bias[left];
    else if (KNNType == "zscore") {
        prediction *= StdDevs[left];
        prediction += Means[left];
    }
    return prediction;
}

// ---------------------------------------------------------------------------------------------
// sim.go on the device

static double sim_pair(Sim kind, const std::vector<IDRating>& a, const std::vector<IDRating>& b) {
    thread_local std::shared_ptr<rs_ctx> ctx;
    if (!ctx) {
        rs_ctx* c = nullptr;
        if (rs_open(0, &c) != RS_OK) panic_rs(nullptr, "rs_open");
        ctx = std::shared_ptr<rs_ctx>(c, rs_close);
    }
    std::vector<int32_t> ai, bi;
    std::vector<double> ar, br;
    for (const auto& x : a) { ai.push_back(x.ID); ar.push_back(x.Rating); }
    for (const auto& x : b) { bi.push_back(x.ID); br.push_back(x.Rating); }
    double out = 0.0;
    if (rs_sim_pair(ctx.get(), static_cast<int32_t>(kind), static_cast<int64_t>(ai.size()), ai.data(),
                    ar.data(), static_cast<int64_t>(bi.size()), bi.data(), br.data(), &out) != RS_OK)
        panic_rs(ctx.get(), "Sim");
    return out;
}
double Cosine(const std::vector<IDRating>& a, const std::vector<IDRating>& b) { return sim_pair(Sim::Cosine, a, b); }
double MSD(const std::vector<IDRating>& a, const std::vector<IDRating>& b) { return sim_pair(Sim::MSD, a, b); }
double Pearson(const std::vector<IDRating>& a, const std::vector<IDRating>& b) { return sim_pair(Sim::Pearson, a, b); }

// ---------------------------------------------------------------------------------------------
// utils.go:160-180, eval.go:18-67

double RMSE(Estimator& e, const DataSet& test) {
    double sum = 0.0;
    for (int64_t j = 0; j < test.Length(); ++j) {
        const double d = e.Predict(test.Users[j], test.Items[j]) - test.Ratings[j];
        sum += d * d;
    }
    return std::sqrt(sum / static_cast<double>(test.Length()));
}

double MAE(Estimator& e, const DataSet& test) {
    double sum = 0.0;
    for (int64_t j = 0; j < test.Length(); ++j)
        sum += std::fabs(e.Predict(test.Users[j], test.Items[j]) - test.Ratings[j]);
    return sum / static_cast<double>(test.Length());
}

std::vector<CrossValidateResult> CrossValidate(const Estimator& estimator, const DataSet& dataSet,
                                               const std::vector<Evaluator>& metrics, int cv,
                                               uint64_t seed, const Parameters& params, int nJobs) {
    std::vector<CrossValidateResult> ret(metrics.size());
    for (auto& r : ret) {
        r.Trains.assign(cv, 0.0);
        r.Tests.assign(cv, 0.0);
    }
    std::vector<int64_t> perm(dataSet.Length());
    std::iota(perm.begin(), perm.end(), 0);
    std::mt19937_64 g(seed);
    std::shuffle(perm.begin(), perm.end(), g);  // data.go:53 rand.Perm (injected seed, Q4)
    std::vector<TrainSet> trains;
    std::vector<DataSet> tests;
    dataSet.KFold(cv, perm, trains, tests);
    const int jobs = nJobs > 0 ? std::min(nJobs, cv) : cv;
    std::vector<std::exception_ptr> err(static_cast<size_t>(jobs));
    std::vector<std::thread> th;
    for (int job = 0; job < jobs; ++job)
        th.emplace_back([&, job] {  // utils.go:145-157: one goroutine per job
            try {
                std::unique_ptr<Estimator> cp = estimator.Clone();  // eval.go:29-30
                for (int i = cv * job / jobs; i < cv * (job + 1) / jobs; ++i) {
                    cp->SetParams(params);  // eval.go:34: params replace the copy's
                    cp->Fit(trains[i]);
                    for (size_t j = 0; j < metrics.size(); ++j) ret[j].Tests[i] = metrics[j](*cp, tests[i]);
                }
            } catch (...) {
                err[job] = std::current_exception();
            }
        });
    for (std::thread& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    return ret;
}

}  // namespace core
