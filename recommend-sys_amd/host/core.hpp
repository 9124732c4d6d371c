// core.hpp -- C++ host mirror of the reference's Go `core` package API for the hot path
// (Oneaccount1/recommend-sys core/base.go, data.go, svd.go, knn.go, sim.go, utils.go, eval.go),
// built on the C-ABI of include/rsgpu.h.  Same names, argument meaning and error behaviour as the
// Go package: Fit has no error return and panics (here: throws core::Panic) on failure, exactly
// where the reference panics or log.Fatal()s; fitted state lives in public fields so Predict runs on
// the host like the reference's.
#pragma once

#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <variant>
#include <vector>

#include "rsgpu.h"

namespace core {

struct Panic : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// sim.go:7 `type Sim func(SortedIdRatings, SortedIdRatings) float64`: the three exported functions
// are identified by kind (Go funcs are not comparable; the cgo binding maps the pointer the same way).
enum class Sim { Cosine = RS_SIM_COSINE, MSD = RS_SIM_MSD, Pearson = RS_SIM_PEARSON };

// base.go:14-57 `Parameters map[string]interface{}` with typed getters; a getter on a value of the
// wrong type panics like the Go type assertion.
using Value = std::variant<int, double, bool, std::string, Sim>;
struct Parameters : std::map<std::string, Value> {
    using std::map<std::string, Value>::map;
    Parameters Copy() const { return *this; }
    int GetInt(const std::string& name, int def) const { return get<int>(name, def); }
    bool GetBool(const std::string& name, bool def) const { return get<bool>(name, def); }
    double GetFloat64(const std::string& name, double def) const { return get<double>(name, def); }
    std::string GetString(const std::string& name, const std::string& def) const {
        return get<std::string>(name, def);
    }
    Sim GetSim(const std::string& name, Sim def) const { return get<Sim>(name, def); }

   private:
    template <typename T>
    T get(const std::string& name, T def) const {
        auto it = find(name);
        if (it == end()) return def;
        if (const T* v = std::get_if<T>(&it->second)) return *v;
        throw Panic("interface conversion: parameter " + name + " has the wrong type");
    }
};

struct IDRating {  // data.go:124-127
    int ID;
    double Rating;
};

constexpr int newID = -1;  // data.go:129

// data.go:21-25 COO of outer ids.
struct DataSet {
    std::vector<double> Ratings;
    std::vector<int64_t> Users, Items;
    int64_t Length() const { return static_cast<int64_t>(Ratings.size()); }
    DataSet SubSet(const std::vector<int64_t>& indices) const;  // data.go:42-47
    // data.go:49-70 with an injected permutation (the reference's rand.Perm is unseeded, Q4)
    void KFold(int k, const std::vector<int64_t>& perm, std::vector<struct TrainSet>& trains,
               std::vector<DataSet>& tests) const;
};

// data.go:109-122 / 131-154: inner ids by first appearance (users, then items).
struct TrainSet : DataSet {
    double GlobalMean = 0.0;
    int UserCount = 0, ItemCount = 0;
    std::unordered_map<int64_t, int> InnerUserIDs, InnerItemIDs;
    std::vector<int32_t> innerUsers, innerItems;  // per rating, cached for the C-ABI
    int ConvertUserID(int64_t userID) const;     // data.go:171-176
    int ConvertItemID(int64_t itemID) const;     // data.go:177-182
    const std::vector<std::vector<IDRating>>& UserRatings() const;  // data.go:185-199
    const std::vector<std::vector<IDRating>>& ItemRatings() const;  // data.go:202-216
    rs_ratings ratings_view(std::vector<double>& r_scratch) const;

   private:
    mutable std::vector<std::vector<IDRating>> userRatings, itemRatings;
};
TrainSet NewTrainSet(const DataSet& raw);
DataSet LoadDataFromFile(const std::string& path, const std::string& sep);  // data.go:287-310 (float ratings, Q10)

// base.go:8-12
class Estimator {
   public:
    Estimator() = default;
    // A copy (Clone) carries Params and Data but opens its own context and RNG stream.
    Estimator(const Estimator& o) : Params(o.Params), Data(o.Data) {}
    Estimator& operator=(const Estimator&) = delete;
    virtual ~Estimator() = default;
    virtual void SetParams(const Parameters& p) { Params = p; }
    virtual double Predict(int64_t userID, int64_t itemID) = 0;
    virtual void Fit(const TrainSet& trainSet) = 0;
    virtual std::unique_ptr<Estimator> Clone() const = 0;  // eval.go:29-30 reflect.New + Copy
    Parameters Params;
    TrainSet Data;

   protected:
    rs_ctx* context();  // lazily opened on Parameters "device" (default 0); never copied
    std::shared_ptr<rs_ctx> ctx_;
    std::vector<double> normal_vector(int n, double mean, double std);  // utils.go:71-77
    std::vector<double> uniform_vector(int n, double low, double high); // utils.go:79-86
    std::mt19937_64& rng();

   private:
    std::unique_ptr<std::mt19937_64> rng_;
};

// svd.go:18-132.  Parameters: nFactors 100, nEpochs 20, lr 0.005, reg 0.02, initMean 0,
// initStdDev 0.1; build extras: "mode" ("fast" | "ordered"), "seed", "device".
class SVD : public Estimator {
   public:
    std::vector<std::vector<double>> UserFactor, ItemFactor;
    std::vector<double> UserBias, ItemBias;
    double GlobalBias = 0.0;
    double Predict(int64_t userID, int64_t itemID) override;
    void Fit(const TrainSet& trainSet) override;
    std::unique_ptr<Estimator> Clone() const override { return std::make_unique<SVD>(*this); }
};
std::unique_ptr<SVD> NewSVD(const Parameters& params = {});

// svd.go:259-433.  nFactors 20, nEpochs 20, lr 0.007, reg 0.02.
class SVDPP : public Estimator {
   public:
    std::vector<std::vector<IDRating>> UserRatings;
    std::vector<std::vector<double>> UserFactor, ItemFactor, ImplFactor;
    std::vector<double> UserBias, ItemBias;
    double GlobalBias = 0.0;
    double Predict(int64_t userID, int64_t itemID) override;
    void Fit(const TrainSet& trainSet) override;
    std::unique_ptr<Estimator> Clone() const override { return std::make_unique<SVDPP>(*this); }
};
std::unique_ptr<SVDPP> NewSVDpp(const Parameters& params = {});

// svd.go:134-257.  nFactors 15, nEpochs 50, initLow 0, initHigh 1, reg 0.06; build extra
// "asWritten" (default true: svd.go:243-249 as written, Q5).
class NMF : public Estimator {
   public:
    std::vector<std::vector<double>> userFactor, itemFactor;
    double Predict(int64_t userID, int64_t itemID) override;
    void Fit(const TrainSet& trainSet) override;
    std::unique_ptr<Estimator> Clone() const override { return std::make_unique<NMF>(*this); }
};
std::unique_ptr<NMF> NewNMF(const Parameters& params = {});

// knn.go:17-217.  Parameters: sim (MSD), userBased (true), k (40), mink (1); the KNN type is the
// constructor's default whatever Params says (Q9, knn.go:50-73).
class KNN : public Estimator {
   public:
    explicit KNN(std::string type) : KNNType(std::move(type)) {}
    std::string KNNType;
    double GlobalMean = 0.0;
    std::vector<double> Sims;  // L x L row-major (Sims[i][j] = Sims[i * L + j]); NaN = no co-rating
    int L = 0;
    std::vector<std::vector<IDRating>> LeftRatings, RightRatings;
    std::vector<double> Means, StdDevs, Bias;
    double Predict(int64_t userID, int64_t itemID) override;
    void Fit(const TrainSet& trainSet) override;
    std::unique_ptr<Estimator> Clone() const override { return std::make_unique<KNN>(*this); }
};
std::unique_ptr<KNN> NewKNN(const Parameters& params = {});
std::unique_ptr<KNN> NewKNNWithMean(const Parameters& params = {});
std::unique_ptr<KNN> NewKNNWithZScore(const Parameters& params = {});
std::unique_ptr<KNN> NewKNNBaseLine(const Parameters& params = {});

// sim.go:10-81 on the device (rs_sim_pair); inputs ID-ascending (SortedIdRatings).
double Cosine(const std::vector<IDRating>& a, const std::vector<IDRating>& b);
double MSD(const std::vector<IDRating>& a, const std::vector<IDRating>& b);
double Pearson(const std::vector<IDRating>& a, const std::vector<IDRating>& b);

// utils.go:160-180 (Evaluator(Estimator, DataSet)).
using Evaluator = std::function<double(Estimator&, const DataSet&)>;
double RMSE(Estimator& e, const DataSet& test);
double MAE(Estimator& e, const DataSet& test);

struct CrossValidateResult {  // eval.go:12-15
    std::vector<double> Trains, Tests;
};
// eval.go:18-67: the cv folds split over nJobs host threads (utils.go:145-157 `parallel`: job j takes folds
// [cv j / nJobs, cv (j + 1) / nJobs)); each job fits its own Clone (eval.go:29-30), which opens its own
// rs_ctx, so the folds' Fits run concurrently on the device (nJobs <= 0: one job per fold)
std::vector<CrossValidateResult> CrossValidate(const Estimator& estimator, const DataSet& dataSet,
                                               const std::vector<Evaluator>& metrics, int cv,
                                               uint64_t seed, const Parameters& params, int nJobs = 0);

}  // namespace core
