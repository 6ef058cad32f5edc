/*
 * fdengine.h — C-ABI of the MI355X-native fraud-scoring engine (libfdengine.so).
 *
 * The engine is the drop-in for ONE hot path of AjayAlluri/realtime-fraud-detection:
 *   windowed per-card features -> XGBoost primary classifier + Isolation Forest anomaly score
 *   -> ensemble blend / decision.
 *
 * Every entry point below replaces a named reference interface (paths relative to the
 * reference repo root; "ml/" = services/ml-models/src/, "fl/" = services/flink-jobs/src/main/
 * java/com/frauddetection/).  The Python host shim (realtime-fraud-detection_amd/fdengine/)
 * binds these with ctypes; INTEGRATION.md shows the binding a maintainer adds.
 *
 * Conventions (mirroring ml/models/model_manager.py:279-307):
 *   - every function returns int status, FD_OK == 0; nothing throws across the ABI;
 *   - fd_last_error() returns a thread-local message for the last failure on this thread;
 *   - caller-owned buffers; "_device" functions take device pointers (HBM-resident inputs),
 *     "_host" functions take host pointers and are synchronous;
 *   - one engine per GPU; every entry point taking an engine holds that engine's (recursive) lock, so
 *     calls from several host threads are serialised per engine (the reference serialises on one
 *     asyncio loop, ml/main.py:337-344; here ModelManager.predict runs in a worker thread beside the
 *     loop's own calls). fd_engine_destroy while another thread still uses the engine is undefined.
 * No PyTorch / HIP types appear in these signatures; streams are passed as void*.
 */
#ifndef FDENGINE_H
#define FDENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FD_ABI_VERSION 15

enum fd_status {
  FD_OK = 0,
  FD_ERR_INVALID_ARG = 1,
  FD_ERR_HIP = 2,
  FD_ERR_NOT_LOADED = 3, /* ValueError("Model ... not loaded"), ml/models/model_manager.py:281-282 */
  FD_ERR_UNSUPPORTED = 4,
  FD_ERR_OOM = 5,
  FD_ERR_IO = 6, /* snapshot file missing / truncated / corrupt (checksum) */
};

/* Forest kinds: the two tree model types on the path. */
enum fd_forest_kind {
  /* xgboost 2.0.3 gbtree, objective binary:logistic
     (ml/models/model_manager.py:157-161 load, :309-311 predict_proba[:,1]) */
  FD_FOREST_XGB_BINARY_LOGISTIC = 1,
  /* scikit-learn IsolationForest, decision_function then 1/(1+e^s)
     (ml/models/model_manager.py:197-200 load, :338-346 predict) */
  FD_FOREST_SKLEARN_IFOREST = 2,
};

typedef struct fd_engine fd_engine;

/* Original (un-repacked) tree arrays of one forest, concatenated over trees.
   Node ids are per tree, 0-based, exactly as the source library numbers them
   (XGBoost JSON `left_children`/... arrays; sklearn `tree_.children_left`/...). */
typedef struct {
  int32_t n_trees;
  const int64_t* tree_offsets; /* n_trees+1 offsets into the node arrays */
  const int32_t* left;         /* left child, -1 marks a leaf */
  const int32_t* right;        /* right child */
  const int32_t* feature;      /* split column in the caller's feature matrix */
  const double* threshold;     /* split value as the library stores it (XGB: f32 value; sklearn: f64) */
  const uint8_t* default_left; /* missing-value (NaN) direction; NULL = right */
  const double* leaf_value;    /* per node, read at leaves (XGB: leaf weight; IF: depth+c(n)-1) */
} fd_tree_arrays;

typedef struct {
  int32_t kind;        /* enum fd_forest_kind */
  int32_t num_feature; /* model columns (XGB learner_model_param.num_feature / sklearn n_features_in_) */
  double base_score;   /* XGB: learner_model_param.base_score (probability space) */
  double if_offset;    /* IF: offset_ */
  double if_denominator; /* IF: n_estimators * _average_path_length([max_samples]) */
} fd_forest_params;

/* Ensemble blend parameters (ml/models/ensemble_predictor.py:62-73, 252-369). Models are listed
   in the reference's enabled-model order (ml/utils/config.py:128-199). */
#define FD_MAX_MODELS 8
enum fd_blend_strategy { FD_BLEND_WEIGHTED_AVERAGE = 0, FD_BLEND_VOTING = 1, FD_BLEND_STACKING = 2 };
enum fd_decision { FD_APPROVE = 0, FD_REVIEW = 1, FD_DECLINE = 2, FD_APPROVE_WITH_MONITORING = 3 };
enum fd_risk { FD_VERY_LOW = 0, FD_LOW = 1, FD_MEDIUM = 2, FD_HIGH = 3, FD_CRITICAL = 4 };
typedef struct {
  int32_t n_models;
  int32_t strategy;                  /* enum fd_blend_strategy */
  double weight[FD_MAX_MODELS];      /* normalised weights, _get_model_weights :62-73 */
  double conf_mult[FD_MAX_MODELS];   /* _calculate_model_confidence multipliers :331-337 */
  double fraud_threshold;            /* EnsembleConfig.fraud_threshold (0.5) */
  double confidence_threshold;       /* EnsembleConfig.confidence_threshold (0.7) */
} fd_blend_params;

/* ---------------------------------------------------------------- engine lifecycle */
const char* fd_last_error(void);
int fd_abi_version(void);
/* "fdengine-build-id:src=<digest>;flags=<hipcc flags>": SHA-256 (first 128 bits) of the HIP sources, the csrc
   headers and this header the library was built from (fdengine/_buildid.py); the Python loader refuses a
   library whose digest differs from the tree beside it. */
const char* fd_build_id(void);
int fd_device_count(int* out);
/* ModelManager.__init__ (ml/models/model_manager.py:33-45): one engine per GPU. */
int fd_engine_create(int device, fd_engine** out);
int fd_engine_destroy(fd_engine* eng);
/* Launch on a caller stream (hipStream_t as void*). NULL is the device's null (default) stream,
   e.g. PyTorch's default stream, whose handle is 0. fd_engine_reset_stream restores the engine's
   own non-blocking stream. */
int fd_engine_set_stream(fd_engine* eng, void* hip_stream);
int fd_engine_reset_stream(fd_engine* eng);
int fd_engine_sync(fd_engine* eng);

/* ---------------------------------------------------------------- forests (a8, a9) */
/* Replaces _load_xgboost_model (ml/models/model_manager.py:157-161) and _load_sklearn_model
   (:197-200): repacks the original trees into the engine's depth-major layout and uploads them. */
int fd_load_forest(fd_engine* eng, int slot, const fd_forest_params* params, const fd_tree_arrays* trees);
int fd_unload_forest(fd_engine* eng, int slot);

/* Load the reference's XGBoost model FILE unchanged into `slot` (replaces ModelManager._load_xgboost_model,
   services/ml-models/src/models/model_manager.py:157-161: XGBClassifier().load_model(path); the file is
   XGBClassifier.save_model's XGBoost 2.0.3 JSON, model_trainer.py:95-108). Parsed in C++ — a C / C++ / JNI
   host needs no Python — then repacked exactly as fd_load_forest. FD_ERR_IO: unreadable file;
   FD_ERR_UNSUPPORTED: objective other than binary:logistic, booster other than gbtree, multi-class,
   categorical splits or vector leaves; FD_ERR_INVALID_ARG: malformed JSON / tree arrays. */
int fd_load_xgboost_json(fd_engine* eng, int slot, const char* path);

/* Host-only (no device): the same file flattened into caller arrays, the parity hook for the reader.
   Call with trees == NULL to get *n_trees / *n_nodes, then with trees' arrays sized n_trees + 1 (offsets)
   and n_nodes (the rest); params receives kind, num_feature and base_score. */
int fd_xgboost_json_read(const char* path, fd_forest_params* params, int32_t* n_trees, int64_t* n_nodes,
                         fd_tree_arrays* trees);
int fd_forest_info(fd_engine* eng, int slot, int32_t* n_trees, int32_t* depth, int32_t* num_feature);

/* Replaces _predict_xgboost (:309-311) / _predict_sklearn (:338-346) for a batch.
   d_X: n x ld row-major f32 (what XGBoost's DMatrix / sklearn's validate_data cast the f64 vector to).
   d_prob: P(fraud) per row (XGB: f32 sigmoid widened; IF: 1/(1+exp(decision_function))).
   d_raw (optional): XGB margin / IF summed path length.
   d_leaf (optional): n x n_trees original leaf node ids (xgboost pred_leaf / sklearn apply). */
int fd_forest_predict_device(fd_engine* eng, int slot, const float* d_X, int64_t n, int32_t ld,
                             double* d_prob, double* d_raw, int32_t* d_leaf);
int fd_forest_predict_host(fd_engine* eng, int slot, const float* X, int64_t n, int32_t ld,
                           double* prob, double* raw, int32_t* leaf);

/* Host-only repack (no device needed): the layouts fd_load_forest uploads, for layout inspection
   and CPU tests. Call with NULL buffers to query sizes in *info.
   fd_pack_forest_host: threshold layout — per tree a 1-based heap of 2^D {f32 thr, u32 meta}
   records (slot 0 unused, children of slot s at 2s / 2s+1) then 2^D leaf values.
   fd_pack_forest_binned_host: binned layout — every split threshold replaced by its index j in the
   feature's sorted table of distinct thresholds (x < t_j  <=>  bin(x) <= j, bin(x) = #{t <= x}), so a
   node is one u32 (j << 16 | feature * 1024 | default_left); 2^D node words then 2^D leaf values.
   Returns FD_ERR_UNSUPPORTED when a feature has more than 65534 distinct thresholds. */
typedef struct {
  int32_t n_trees;
  int32_t n_chunks;
  int32_t chunk;        /* trees per LDS staging chunk */
  int32_t depth;        /* D: every tree is padded to a perfect depth-D tree */
  int64_t tree_bytes;   /* 2^D node records (8 B threshold layout / 4 B binned) + 2^D leaf values
                           (f32 XGB / f64 IF) */
  int64_t chunk_stride; /* bytes per chunk, 1 KiB multiple */
  int64_t blob_bytes;
  int64_t n_leaf_ids;
  float base_margin;    /* XGB: f32 margin seeded by base_score */
  int32_t layout;       /* 0 threshold layout, 1 binned layout */
  int64_t n_thresholds; /* binned: total distinct thresholds over all features */
  int32_t bin_steps;    /* binned: largest power of two <= the longest feature table (0 if none) */
} fd_pack_info;
int fd_pack_forest_host(const fd_forest_params* params, const fd_tree_arrays* trees, void* blob,
                        int64_t blob_cap, int32_t* leaf_ids, int64_t ids_cap, fd_pack_info* info);
/* thresholds: n_thresholds f32 (feature-major, ascending per feature); offsets: num_feature + 1. */
int fd_pack_forest_binned_host(const fd_forest_params* params, const fd_tree_arrays* trees, void* blob,
                               int64_t blob_cap, float* thresholds, int64_t thr_cap, int32_t* offsets,
                               fd_pack_info* info);

/* ---------------------------------------------------------------- blend (a11-a13) */
/* Replaces _calculate_model_confidence + _combine_predictions + _make_decision +
   _calculate_risk_level (ml/models/ensemble_predictor.py:252-369) for a batch.
   d_probs[m] (host array of device pointers) is model m's probability column; present[m] == 0
   drops model m as a failed prediction is dropped (:175-181). */
int fd_blend_device(fd_engine* eng, const fd_blend_params* params, int64_t n,
                    const double* const* d_probs, const uint8_t* present,
                    double* d_fraud_prob, double* d_confidence, uint8_t* d_decision, uint8_t* d_risk);
int fd_blend_host(fd_engine* eng, const fd_blend_params* params, int64_t n,
                  const double* const* probs, const uint8_t* present,
                  double* fraud_prob, double* confidence, uint8_t* decision, uint8_t* risk);

/* ---------------------------------------------------------------- card state + features (a2-a7) */
/* HBM-resident keyed state replacing the Redis round trips of the feature half:
   velocity hashes velocity:{user}:{5min|1hour|24hour} (fl/services/RedisService.java:178-207,
   fl/sinks/RedisTransactionSink.java:116-135) and the user-profile lookups (RedisService.java:83-100).
   Cards are keyed by a u64 (hash of the reference's user_id); open addressing, insert on first use. */
enum fd_window_mode {
  FD_WINDOW_REDIS_COMPAT = 0, /* session counter, TTL 3600 s refreshed per write: the reference's behaviour */
  FD_WINDOW_SLIDING = 1       /* true (t-W, t] windows over the card's last ring_k events */
};
#define FD_RAW_FEATURES 16  /* bridged Flink features per txn (column order: DESIGN.md "Features") */
#define FD_VECTOR_WIDTH 64  /* EnsemblePredictor._prepare_features width (ml/models/ensemble_predictor.py:241) */
#define FD_MAX_SEQ_LEN 16
typedef struct {
  int64_t capacity;    /* card slots (rounded up to a power of two; keep >= 2x the cards expected) */
  int32_t window_mode; /* enum fd_window_mode */
  int32_t ring_k;      /* events kept per card in sliding mode (1..64) */
  int32_t seq_len;     /* events of per-card history kept for the LSTM head (0 = off, <= 16;
                          lstm_sequential sequence_length = 10, ml/utils/config.py:152) */
} fd_state_params;
int fd_state_init(fd_engine* eng, const fd_state_params* params);
int fd_state_clear(fd_engine* eng);
int fd_state_info(fd_engine* eng, int64_t* capacity, int64_t* cards);
/* user profiles (simulator.py:40-58 UserProfile; FeatureExtractor.java:216-252, 301-313) */
typedef struct {
  int64_t n;
  const uint64_t* key;
  const double* avg_amount;        /* NaN = null (-> 0.0, FeatureExtractor.java:239-240) */
  const int32_t* account_age_days;
  const uint64_t* device_fp;       /* n x 3 fingerprint hashes, 0 = none */
} fd_users;
int fd_state_load_users_host(fd_engine* eng, const fd_users* users);
/* merchant table, replicated (simulator.py:60-75; FeatureExtractor.java:257-296) */
typedef struct {
  int64_t n;
  const double* fraud_rate;      /* NaN = null (-> 0.05) */
  const double* risk_multiplier; /* MerchantProfile.getRiskMultiplier() (class absent in the reference) */
} fd_merchants;
int fd_load_merchants_host(fd_engine* eng, const fd_merchants* merchants);
/* one micro-batch of transactions in arrival order (SoA; device pointers for _device, host for _host) */
typedef struct {
  const uint64_t* card_key;
  const int64_t* ts_ms;
  const int64_t* amount_cents;
  const int32_t* merchant;   /* index into the merchant table, -1 = unknown */
  const uint64_t* device_fp; /* 0 = null */
  const uint8_t* ip_class;   /* 0 = null, 1 = private, 2 = public (FeatureExtractor.java:434-445) */
  const uint8_t* hour;       /* Transaction.hourOfDay, 255 = null (-> UTC hour of ts) */
  const uint8_t* weekend;    /* Transaction.isWeekend, 255 = null (-> ISO day >= 6) */
} fd_txn_batch;
/* Replaces FeatureExtractor.extractAllFeatures + the velocity read/write + FeatureProcessor +
   _prepare_features for a batch: per card in arrival order, read-before-write. Outputs the scoring
   vectors (n x 64 f32) and optionally the bridged raw features (n x FD_RAW_FEATURES f64). */
int fd_features_device(fd_engine* eng, const fd_txn_batch* txns, int64_t n, float* d_vectors, double* d_raw);
int fd_features_host(fd_engine* eng, const fd_txn_batch* txns, int64_t n, float* vectors, double* raw);

/* ---------------------------------------------------------------- full feature map + rule scores (a3, (f)) */
/* FeatureExtractor.extractAllFeatures as a whole (fl/features/FeatureExtractor.java:50-493): the 64
   features of FeatureStore.getRegisteredFeatures (fl/features/FeatureStore.java:325-365, that order),
   f64, NaN where the Java map would have no key; string features as the host's vocabulary codes
   (FD_CODE_UNKNOWN for the literal "unknown"). Plus the Flink rule scores that consume them:
   FeatureEnrichmentProcessor (calculateFeatureBasedFraudScore, combine with the incoming score,
   updateRiskLevel; fl/processors/FeatureEnrichmentProcessor.java:80-93,122-367) and TransactionProcessor
   (calculateBasicFeatures, applyFraudDetectionRules, makeFinalDecision with minimal profiles for
   unknown users / merchants; fl/processors/TransactionProcessor.java:143-508). */
#define FD_FEATURE_MAP_WIDTH 64
#define FD_CODE_UNKNOWN 254
/* per-transaction context beyond fd_txn_batch; any pointer may be NULL (= all null) */
typedef struct {
  const double* geo_lat;          /* Transaction.geolocation lat / lon, NaN = absent */
  const double* geo_lon;
  const double* merchant_lat;     /* Transaction.merchantLocation lat / lon, NaN = absent */
  const double* merchant_lon;
  const uint8_t* payment_method;  /* vocabulary code, 255 = null */
  const uint8_t* transaction_type;
  const uint8_t* card_type;
  const uint8_t* user_agent_flag; /* analyzeSuspiciousUserAgent (host-side string test), 255 = null UA */
  const double* fraud_score;      /* incoming Transaction.fraudScore, NaN = null */
} fd_txn_context;
typedef struct {
  double tp_score;      /* TransactionProcessor fraud score */
  double fe_score;      /* FeatureEnrichmentProcessor fraud score */
  uint8_t tp_decision;  /* enum fd_decision */
  uint8_t tp_risk;      /* enum fd_risk */
  uint8_t fe_decision;
  uint8_t fe_risk;
  uint8_t pad[4];
} fd_rule_scores;
/* UserProfile fields beyond fd_users (simulator.py:40-58); keyed like fd_users; NULL arrays = null */
typedef struct {
  int64_t n;
  const uint64_t* key;
  const double* risk_score;        /* NaN = null */
  const uint8_t* kyc_status;       /* vocabulary code, 255 = null */
  const uint8_t* verified;         /* UserProfile.isVerified() */
  const int8_t* pref_start;        /* preferred hours, -1 = null */
  const int8_t* pref_end;
  const double* weekend_activity;  /* behavioral pattern values, NaN = absent */
  const double* online_preference;
  const double* intl_preference;   /* international_transactions, NaN = null */
  const int32_t* txn_frequency;    /* -1 = null */
  const uint8_t* has_patterns;     /* getBehavioralPatterns() != null */
} fd_users_ext;
/* MerchantProfile fields beyond fd_merchants (simulator.py:60-75), indexed like fd_merchants */
typedef struct {
  int64_t n;
  const double* avg_amount;           /* NaN = null */
  const uint8_t* risk_level;          /* 0 low, 1 medium, 2 high (vocabulary), 255 = null */
  const uint8_t* blacklisted;         /* 255 = null */
  const uint8_t* category;            /* vocabulary code, 255 = null */
  const uint8_t* high_risk_category;  /* MerchantProfile.isHighRiskCategory() */
  const uint8_t* open_hour;           /* operating hours [open, close), 255 = null */
  const uint8_t* close_hour;
  const uint8_t* suspicious_name;     /* analyzeMerchantName (host regexes), 255 = null name */
} fd_merchants_ext;
int fd_state_load_users_ext_host(fd_engine* eng, const fd_users_ext* users);
int fd_load_merchants_ext_host(fd_engine* eng, const fd_merchants_ext* merchants);
/* 256 flags each: payment-method code -> isHighRiskPaymentMethod, transaction-type code -> "refund" */
int fd_load_vocab_host(fd_engine* eng, const uint8_t* payment_high_risk, const uint8_t* type_is_refund);
/* fd_features_* plus the feature map (n x FD_FEATURE_MAP_WIDTH f64) and rule scores; d_fmap / d_rules /
   d_raw may be NULL. Advances the card state exactly like fd_features_device. */
int fd_features_full_device(fd_engine* eng, const fd_txn_batch* txns, const fd_txn_context* ctx, int64_t n,
                            float* d_vectors, double* d_raw, double* d_fmap, fd_rule_scores* d_rules);

/* ---------------------------------------------------------------- LSTM sequence head (a10) */
/* Replaces _load_tensorflow_model / _predict_tensorflow (ml/models/model_manager.py:162-165, 313-319)
   for lstm_sequential (ml/utils/config.py:145-157). Model: 1-layer LSTM(hidden = 128) over a sequence
   of per-event inputs (input_size <= 16), gates in Keras / PyTorch order i, f, g, o, then a dense head:
   n_out = 1 -> sigmoid(z), n_out = 2 -> softmax(z)[1] (_predict_tensorflow takes [:, 1] when the output
   has 2 columns, else flattens). Weights in PyTorch layout, f32 (the host converts Keras kernels):
   w_ih [4H x input_size], w_hh [4H x H], b_ih / b_hh [4H] (either may be NULL), w_out [n_out x H],
   b_out [n_out]. Computed in f32 on the matrix cores. */
typedef struct {
  int32_t input_size;
  int32_t hidden;
  int32_t n_out;
  const float* w_ih;
  const float* w_hh;
  const float* b_ih;
  const float* b_hh;
  const float* w_out;
  const float* b_out;
} fd_lstm_params;
int fd_load_lstm(fd_engine* eng, const fd_lstm_params* params);
int fd_unload_lstm(fd_engine* eng);
/* d_seq: n x T x 16 f32 (events oldest -> newest, inputs beyond input_size ignored); d_prob: n f64 */
int fd_lstm_predict_device(fd_engine* eng, const float* d_seq, int64_t n, int32_t T, double* d_prob);
int fd_lstm_predict_host(fd_engine* eng, const float* seq, int64_t n, int32_t T, double* prob);
/* In fd_score_batch_device / fd_score_records_device, a model whose slot is FD_SLOT_LSTM is the LSTM head
   over each transaction's card history (the last seq_len events including itself, fd_state_params.seq_len
   > 0); it runs on a second stream concurrently with the forests. fd_features_seq_device also returns
   those sequences (n x seq_len x 16 f32). */
#define FD_SLOT_LSTM 64
int fd_features_seq_device(fd_engine* eng, const fd_txn_batch* txns, int64_t n, float* d_vectors, double* d_raw,
                           float* d_seq);

/* ---------------------------------------------------------------- batched scoring */
/* Replaces the per-transaction loop of /batch-predict (ml/main.py:235-249) for prepared scoring
   vectors: every forest model scores the same X, then the blend runs, all on the device.
   Model m (blend order) is either a loaded forest (slots[m] >= 0) or an externally computed
   probability column ext_probs[m] (slots[m] < 0; host pointer for _host, device for _device);
   present[m] == 0 drops model m. d_model_probs (optional) receives the n x n_models column-major
   per-model probabilities (model m at offset m*n). */
int fd_score_matrix_device(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                           const double* const* ext_probs, const uint8_t* present, const float* d_X,
                           int64_t n, int32_t ld, double* d_model_probs, double* d_fraud_prob,
                           double* d_confidence, uint8_t* d_decision, uint8_t* d_risk);
int fd_score_matrix_host(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                         const double* const* ext_probs, const uint8_t* present, const float* X, int64_t n,
                         int32_t ld, double* model_probs, double* fraud_prob, double* confidence,
                         uint8_t* decision, uint8_t* risk);

/* The whole hot path for one micro-batch of transactions: fd_features_* (card state read/update,
   scoring vectors) then fd_score_matrix_* on those vectors (ld = FD_VECTOR_WIDTH). d_vectors may be
   NULL (engine scratch). Equivalent to the reference's per-transaction chain
   FeatureExtractor -> RedisTransactionSink -> FeatureProcessor -> EnsemblePredictor.predict. */
int fd_score_batch_device(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                          const double* const* ext_probs, const uint8_t* present, const fd_txn_batch* txns,
                          int64_t n, float* d_vectors, double* d_model_probs, double* d_fraud_prob,
                          double* d_confidence, uint8_t* d_decision, uint8_t* d_risk);

/* Streaming form of fd_score_batch_device for a sequence of micro-batches (the Flink operator chain is
   pipelined record by record; here micro-batch by micro-batch). Same results, same card-state order.
   Batch i's feature and scoring launches run on one of the engine's two private pipeline streams
   (alternating by batch), the features ordered after batch i-1's feature launches and after
   `input_ready` (a hipEvent_t the caller recorded once the batch's input columns were in device memory;
   NULL = they were complete before this call). Batch i+1's features therefore overlap batch i's forests.
   The scoring launches write engine-owned staging; the caller's output buffers are written by one copy
   kernel queued on the ENGINE stream (fd_engine_set_stream) after batch i's scoring: the outputs are
   ordered on the engine stream exactly as with fd_score_batch_device, and a caller may free or reuse
   them in that stream's order (e.g. torch's caching allocator on the stream the engine is bound to).
   d_vectors (optional, n x FD_VECTOR_WIDTH f32) receives the batch's scoring vectors the same way.
   The input columns must stay unchanged until the engine stream has passed the call (the engine stream
   waits for the batch's features and scoring). Any other engine call in between orders the next
   batch's features after everything queued on the engine stream (no overlap across it). */
int fd_score_batch_pipelined(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                             const double* const* ext_probs, const uint8_t* present, const fd_txn_batch* txns,
                             int64_t n, float* d_vectors, double* d_model_probs, double* d_fraud_prob,
                             double* d_confidence, uint8_t* d_decision, uint8_t* d_risk, void* input_ready);

/* per-transaction window / sink inputs beyond fd_txn_batch; any pointer may be NULL */
typedef struct fd_window_inputs_s {
  const uint8_t* payment_method; /* vocabulary code, 255 = null (NULL: all null) */
  const uint8_t* is_fraud;       /* Transaction.isFraud, nonzero = TRUE (NULL: all false) */
  const double* fraud_score;     /* Transaction.fraudScore, NaN = null (NULL: all null) */
} fd_window_inputs;

/* ---------------------------------------------------------------- card-hash sharding */
/* The reference partitions per-card work by key (Kafka key / Flink keyBy(userId),
   fl/FraudDetectionJob.java; velocity state in one Redis, fl/services/RedisService.java:178-207).
   Here GPU r of G owns the cards with fd_shard_of(card_key, G) == r and keeps their state in its HBM.
   One micro-batch step on G GPUs (the host shim drives the two RCCL all-to-alls):
     ingest GPU : fd_route_partition_device   -> records grouped by owner (stable) + per-owner counts
     (all-to-all of counts, then of FD_ROUTE_RECORD_BYTES records)
     owner GPU  : fd_score_records_device      -> features + forests + blend, FD_RESULT_RECORD_BYTES records
     (all-to-all of result records back, reversed splits)
     ingest GPU : fd_route_scatter_results_device -> results in the micro-batch's original order.
   Records from one source keep their arrival order, so every card sees its transactions in
   (step, ingest rank, ingest index) order. */
#define FD_MAX_SHARDS 64
#define FD_ROUTE_RECORD_BYTES 48
#define FD_RESULT_RECORD_BYTES 24
/* owner shard of each key (host-only; what the shim uses to load each GPU's user profiles) */
int fd_shard_of_host(const uint64_t* keys, int64_t n, int32_t n_shards, int32_t* out);
/* d_records: n x FD_ROUTE_RECORD_BYTES, owner-major, stable; d_counts: n_shards int64 (device) */
int fd_route_partition_device(fd_engine* eng, const fd_txn_batch* txns, int64_t n, int32_t n_shards,
                              void* d_records, int64_t* d_counts);
/* same, the records also carrying the window / sink inputs the owner needs (extra may be NULL; its
   payment_method and is_fraud are read, fraud_score is produced by the owner) */
int fd_route_partition_ex_device(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* extra,
                                 int64_t n, int32_t n_shards, void* d_records, int64_t* d_counts);
/* the same on the caller's `stream` (a hipStream_t; its own scratch), leaving the engine stream and the
   pipelined stream undisturbed: the pipelined sharded step partitions the next micro-batch and exchanges its
   counts while the owner GPUs still score the current one (fdengine/sharding.py) */
int fd_route_partition_stream(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* extra,
                              int64_t n, int32_t n_shards, void* d_records, int64_t* d_counts, void* stream);
/* owner side: received records (+ their result records, may be NULL) back to columns for the window /
   sink kernels: out's non-NULL fields (card_key, ts_ms, amount_cents, merchant, device_fp, ip_class, hour,
   weekend) and payment_method / is_fraud / fraud_score (the result's fraud_prob; NaN without results) */
int fd_route_unpack_device(fd_engine* eng, const void* d_records, const void* d_results, int64_t n,
                           const fd_txn_batch* out, uint8_t* d_payment_method, uint8_t* d_is_fraud,
                           double* d_fraud_score);
/* the whole hot path (fd_score_batch_device) over received records; d_results: n x FD_RESULT_RECORD_BYTES
   {f64 fraud_prob, f64 confidence, u32 seq, u8 decision, u8 risk, u16 pad} in the records' order */
int fd_score_records_device(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                            const uint8_t* present, const void* d_records, int64_t n, void* d_results);
/* streaming form over received records (fd_score_batch_pipelined's pipeline: features on the engine's
   pipeline streams after the previous batch's features and after `input_ready` — the event the caller
   recorded once the records' all-to-all had landed —, scoring, then d_results written on the engine
   stream, where the caller queues the return all-to-all). The owner's batch i+1 features overlap batch i's
   forests; the records must stay unchanged until the engine stream has passed the call. */
int fd_score_records_pipelined(fd_engine* eng, const fd_blend_params* params, const int32_t* slots,
                               const uint8_t* present, const void* d_records, int64_t n, void* d_results,
                               void* input_ready);
/* The sharded step as one call over the engine's own RCCL communicators (csrc/comm.hip): the host loads
   RCCL once (the process's librccl.so, by path; any library exporting ncclGetUniqueId, ncclCommInitRank,
   ncclCommDestroy, ncclCommAbort, ncclGroupStart/End, ncclSend/Recv, ncclAllGather and ncclGetErrorString can stand in — the tests run several
   ranks on one GPU over an in-process loopback of that API), rank 0 makes two unique ids (fd_comm_unique_id), the
   host broadcasts them, every rank calls fd_comm_init (collective, blocking with RCCL). fd_sharded_step then runs
   one micro-batch: its split sizes (exchanged by the previous call when it prefetched this batch, else now: the
   step's one host wait), then, on the engine's forward stream behind the wait for this batch's inbox slot, ONE
   RCCL group holding this batch's records to their owners (ncclSend/ncclRecv with per-peer counts) and — with
   `next` (optional: prefetch) — the next batch's count exchange (from 4 ranks one ncclAllGather of every rank's
   per-peer send counts right after the group, below that 2 x world point-to-point operations inside it: engine
   option count_exchange), its
   count kernel queued before the group and its publish + places after it (so the next counts land while this
   batch is scored), then the owner's
   features + scoring (fd_score_records_pipelined's pipeline, the features waiting for the records), the
   results back (second communicator, engine stream) and into arrival order in the caller's outputs (device or
   host-mapped memory), written on the engine stream. The calling thread issues every communicator operation, in
   one fixed order; every rank makes the same calls in the same order (the same prefetch pattern).
   Batch ids (caller-chosen): `next_id` (nonzero) names the prefetched batch; the call that scores it passes the
   same id as `batch_id`. batch_id 0 means "not the prefetched batch": a pending prefetch is dropped (its count
   exchange completes, its records are never sent — every rank must drop alike). A nonzero batch_id that is not
   the pending one (or with nothing pending) fails with FD_ERR_INVALID_ARG and changes nothing. The caller keeps a prefetched batch's input
   columns alive and unchanged until the call that scores (or drops) it has returned.
   split_sizes (optional): the 2 x world send / receive counts of this batch.
   Failure: the split-size wait gives up after the engine option comm_timeout_ms (a peer that never posts its counts)
   or on a stream error; it first aborts both communicators (ncclCommAbort: RCCL's kernels blocked on the peer exit),
   then fails with FD_ERR_HIP. Later fd_sharded_step calls fail with the abort's reason; fd_engine_sync,
   fd_comm_destroy and fd_engine_destroy wait on the streams at most comm_timeout_ms each; fd_comm_destroy then
   fd_comm_init makes new communicators. */
int fd_comm_unique_id(const char* rccl_path, uint8_t* id_out /* 128 bytes */);
int fd_comm_init(fd_engine* eng, const char* rccl_path, int32_t rank, int32_t world, const uint8_t* id_fwd,
                 const uint8_t* id_back);
int fd_comm_destroy(fd_engine* eng);
int fd_sharded_step(fd_engine* eng, const fd_blend_params* params, const int32_t* slots, const uint8_t* present,
                    const fd_txn_batch* txns, int64_t n, uint64_t batch_id, void* input_ready,
                    const fd_txn_batch* next, int64_t next_n, uint64_t next_id, void* next_ready,
                    double* d_fraud_prob, double* d_confidence, uint8_t* d_decision, uint8_t* d_risk,
                    int64_t* split_sizes);
/* out[seq] = result for each of the n returned records; conf/decision/risk may be NULL.
   fd_engine_sync reports a record whose seq is outside [0, n). */
int fd_route_scatter_results_device(fd_engine* eng, const void* d_results, int64_t n, double* d_fraud_prob,
                                    double* d_confidence, uint8_t* d_decision, uint8_t* d_risk);

/* ---------------------------------------------------------------- Flink window aggregates (a5) */
/* WindowProcessor.processUserVelocity / processMerchantPatterns (fl/windows/WindowProcessor.java:36-66)
   with UserVelocityAggregateFunction (:248-352) and MerchantAggregateFunction (:357-484), evaluated per
   micro-batch on the device: keyBy(card key) sliding 5 min / slide 1 min, keyBy(merchant) tumbling 1 h,
   event time with BoundedOutOfOrderness watermarks. Micro-batch semantics (DESIGN.md "Windows"): after a
   batch's events are added, the watermark becomes max(previous, max event time - lag - 1) and every window
   whose last millisecond it passed fires once with the events of its range that arrived so far (later
   arrivals are late for it and dropped, allowed lateness 0). Transactions with an unknown merchant (-1)
   are not aggregated by merchant (keyBy on a null id). Amount sums are exact integer cents. */
typedef struct {
  int64_t log_capacity;            /* events kept per log (user / merchant), 40 B each, device-resident */
  int64_t max_out_of_orderness_ms; /* watermark lag: forBoundedOutOfOrderness(10 s) = 10000 */
} fd_window_params;

/* UserVelocityAggregate (getResult :292-311) + the Flink window bounds; 96 B */
typedef struct {
  uint64_t user_key;
  int64_t window_start, window_end; /* Flink TimeWindow [start, end) */
  int64_t first_ts, last_ts;        /* accumulator windowStart / windowEnd: min / max event time (ms) */
  int32_t count, fraud_count, high_risk_count, unique_merchants, unique_payment_methods, pad;
  double total_amount, avg_amount, fraud_rate, velocity_score;
} fd_user_window;
/* MerchantAggregate (getResult :403-424) + the Flink window bounds + the exact moments it is derived from
   (what fd_merchant_windows_merge combines across shards); 168 B */
typedef struct {
  int32_t merchant, count;
  int64_t window_start, window_end, first_ts, last_ts;
  int32_t fraud_count, high_risk_count, unique_users, unique_payment_methods;
  double total_amount, fraud_amount, avg_amount, fraud_rate, amount_stddev, risk_score;
  int64_t cents, fraud_cents;   /* exact amount sums (integer cents) */
  uint64_t sq_lo, sq_hi;        /* sum of cents^2, 128-bit */
  uint64_t pm_mask[4];          /* payment-method codes seen (bit per code) */
} fd_merchant_window;
/* allocate the event logs and reset the watermark (needs fd_state_init: cards are keyed by its table;
   fd_state_init / fd_state_clear empty the logs and reset the watermark too). After a failed step
   (FD_ERR_OOM) the window state is unspecified until the next fd_windows_init. */
int fd_windows_init(fd_engine* eng, const fd_window_params* params);
/* add one micro-batch (device pointers) and return the windows that fired, into host arrays of the given
   capacities (FD_ERR_OOM if more fired); with flush != 0 the watermark then moves past every held event
   (end of input: Flink's final MAX_WATERMARK) and all remaining windows fire. Synchronous. */
int fd_windows_step_device(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* in, int64_t n,
                           int flush, fd_user_window* user_out, int64_t user_cap, int64_t* n_user,
                           fd_merchant_window* merchant_out, int64_t merchant_cap, int64_t* n_merchant);
/* same, host input pointers (staged to the device) */
int fd_windows_step_host(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* in, int64_t n,
                         int flush, fd_user_window* user_out, int64_t user_cap, int64_t* n_user,
                         fd_merchant_window* merchant_out, int64_t merchant_cap, int64_t* n_merchant);
/* current watermark (INT64_MIN before the first) and events held in the user / merchant logs */
int fd_windows_stats(fd_engine* eng, int64_t* watermark, int64_t* user_events, int64_t* merchant_events);
/* Sharded windows: every shard advances ONE watermark — before its step, each shard reports the
   largest event time of the whole node's micro-batch (an all-reduce MAX of the ingest batches); the next step
   then advances the watermark from it even when this shard received no transaction. Each shard's user
   windows are complete (cards are owned); its merchant windows are partials over its cards. */
int fd_windows_observe(fd_engine* eng, int64_t max_event_ts);
/* Merge merchant-window partials of several shards (host memory, any order): records with the same
   (merchant, window_start) are combined from their exact moments (counts, cents, cents^2, payment-method
   set, first / last time; distinct users add: a card lives on one shard) and the derived fields recomputed
   exactly as the device does. out: capacity n; *n_out merged records sorted by (window_start, merchant).
   Host only (no GPU needed). */
int fd_merchant_windows_merge(const fd_merchant_window* parts, int64_t n, fd_merchant_window* out, int64_t* n_out);

/* ---------------------------------------------------------------- sink aggregates */
/* RedisTransactionSink.updateAggregations (fl/sinks/RedisTransactionSink.java:140-262): per transaction the
   hourly:{ts/3600000}, daily:{ts/86400000} and merchant:{merchant}:{ts/3600000} summaries (count, amount,
   fraud count, high-risk count (hourly, fraudScore > 0.7), distinct users (merchant)), HBM-resident.
   Amounts are exact integer cents (reported / 100); the reference's 30-min Redis TTL is wall-clock, so
   retention here is explicit (fd_sink_evict_before). Declared semantics: DESIGN.md §4.8. */
typedef struct {
  int64_t capacity;      /* aggregate entries (hourly + daily + merchant-hour buckets held at once) */
  int64_t user_capacity; /* distinct (merchant, hour, card) members held at once */
} fd_sink_params;
enum fd_agg_kind { FD_AGG_HOURLY = 1, FD_AGG_DAILY = 2, FD_AGG_MERCHANT = 3 };
typedef struct { /* the stored aggregation map (updateHourly/Daily/MerchantAggregations :165-262); 64 B */
  int64_t total_count, fraud_count, high_risk_count, unique_user_count;
  double total_amount, fraud_rate, avg_amount;
  int32_t found, pad;
} fd_aggregate;
int fd_sink_init(fd_engine* eng, const fd_sink_params* params);
/* apply one micro-batch (device pointers; card_key, ts_ms, amount_cents, merchant of fd_txn_batch; is_fraud /
   fraud_score of fd_window_inputs, NULL = false / null). Synchronous (error check). */
int fd_sink_update_device(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* in, int64_t n);
int fd_sink_update_host(fd_engine* eng, const fd_txn_batch* txns, const fd_window_inputs* in, int64_t n);
/* RedisService.getAggregation: bucket = hour or day key, merchant index for FD_AGG_MERCHANT (else ignored) */
int fd_sink_query_host(fd_engine* eng, int32_t kind, const int64_t* bucket, const int32_t* merchant, int64_t n,
                       fd_aggregate* out);
/* drop every bucket older than hour_key (a day is kept while any of its hours is) */
int fd_sink_evict_before(fd_engine* eng, int64_t hour_key, int64_t* kept_entries, int64_t* kept_users);

/* ---------------------------------------------------------------- state snapshot / restore */
/* Durable image of the HBM keyed state: the counterpart of Flink's keyed-state checkpoints
   (fl/FraudDetectionJob.java:112-136) and the Redis RDB of the velocity / profile hashes
   (config/redis/redis-master.conf:6-13). Key-addressed (one record per card: header, fingerprints, ring,
   LSTM history, extended profile), then the replicated merchant / vocabulary tables and the window event
   logs; per-section FNV-1a-64 checksums. Synchronous; written to `path`.tmp then renamed.
   (shard, n_shards) are recorded in the image for bookkeeping (0, 1 for an unsharded engine). */
int fd_state_snapshot(fd_engine* eng, const char* path, int32_t shard, int32_t n_shards, int64_t* bytes_written);
/* Re-insert an image's cards by key into the current table (any capacity; window_mode / ring_k / seq_len
   must match fd_state_init's) keeping only the cards with shard_of(key, n_shards) == shard — restoring
   every old shard's image on every new shard re-shards the state onto a different GPU count. Replicated
   tables are replaced. Window logs are appended (fd_windows_init first) unless FD_RESTORE_SKIP_WINDOWS;
   images merged onto one engine must share the window watermark. The image also carries the sink aggregates
   (replaced on restore; same shard / shard count only, else FD_RESTORE_SKIP_SINK) and the ingest codec's merchant /
   vocabulary tables (replaced). On FD_ERR_IO / FD_ERR_OOM the state is unspecified until fd_state_clear. */
#define FD_RESTORE_SKIP_WINDOWS 1
#define FD_RESTORE_SKIP_SINK 2 /* sink aggregates (fd_sink_*) resume only on the same shard / shard count */
int fd_state_restore(fd_engine* eng, const char* path, int32_t shard, int32_t n_shards, int32_t flags,
                     int64_t* cards_restored);

/* ---------------------------------------------------------------- Kafka JSON ingest codec */
/* TransactionDeserializationSchema.deserialize (fl/serialization/TransactionDeserializationSchema.java:28-49)
   of the simulator's messages (json.dumps(asdict(Transaction), default=str),
   services/data-simulator/src/main/python/simulator.py:77-101,186,376-385) on the device: one micro-batch of
   raw messages (concatenated bytes + n+1 offsets) -> the SoA columns below. Identities: card_key =
   fd_hash64(user_id), device_fp = fd_hash64(device_fingerprint), txn_hash = fd_hash64(transaction_id);
   merchant = index of merchant_id in fd_ingest_set_merchants (-1 unknown / null); payment_method /
   transaction_type / card_type = index in fd_ingest_set_vocab (255 null, FD_VOCAB_OTHER unknown);
   ip_class 0 null / 1 private / 2 public and user_agent_flag 0 / 1 / 255 null (FeatureExtractor.java:434-451);
   ts_ms = ISO-8601 timestamp as epoch ms (UTC without offset); amount_cents exact. Declared semantics and
   limits: DESIGN.md "Ingest". Rows with status & FD_INGEST_INVALID are the reference's ERROR placeholder
   (all other columns default). Any output pointer may be NULL. */
#define FD_VOCAB_OTHER 254
enum fd_vocab_kind { FD_VOCAB_PAYMENT_METHOD = 0, FD_VOCAB_TRANSACTION_TYPE = 1, FD_VOCAB_CARD_TYPE = 2 };
enum fd_ingest_status {
  FD_INGEST_MALFORMED = 1,     /* not one JSON object / bad member syntax / value of the wrong type */
  FD_INGEST_TOO_LONG = 2,      /* message longer than 4080 bytes */
  FD_INGEST_UNKNOWN_VOCAB = 4, /* a payment / type / card string outside its vocabulary (code FD_VOCAB_OTHER) */
  FD_INGEST_INEXACT = 8,       /* sub-cent amount (rounded half-even) or a > 19-digit number at a rounding tie */
  FD_INGEST_MISSING = 16,      /* user_id, amount or timestamp missing / null */
};
#define FD_INGEST_INVALID (FD_INGEST_MALFORMED | FD_INGEST_TOO_LONG | FD_INGEST_MISSING)
typedef struct {
  uint64_t* card_key;
  int64_t* ts_ms;
  int64_t* amount_cents;
  int32_t* merchant;
  uint64_t* device_fp;
  uint8_t* ip_class;
  uint8_t* hour;
  uint8_t* weekend;
  double* geo_lat;
  double* geo_lon;
  double* merchant_lat;
  double* merchant_lon;
  uint8_t* payment_method;
  uint8_t* transaction_type;
  uint8_t* card_type;
  uint8_t* user_agent_flag;
  double* fraud_score;
  uint8_t* is_fraud;
  uint64_t* txn_hash;
  uint8_t* status;
} fd_ingest_out;
/* the identity hash of the codec: fmix64(FNV-1a-64(bytes)) (host; profiles / merchants are keyed with it) */
int fd_hash64(const uint8_t* bytes, int64_t n, uint64_t* out);
/* vocabulary `which` (enum fd_vocab_kind): string i (bytes[offsets[i]..offsets[i+1])) gets code i (n <= 254) */
int fd_ingest_set_vocab(fd_engine* eng, int32_t which, const uint8_t* bytes, const int64_t* offsets, int64_t n);
/* merchant_id strings in merchant-table order (index = the engine's merchant index) */
int fd_ingest_set_merchants(fd_engine* eng, const uint8_t* bytes, const int64_t* offsets, int64_t n);
/* device pointers (HBM-resident messages, outputs); asynchronous on the engine stream; n <= 2^30 */
int fd_ingest_json_device(fd_engine* eng, const uint8_t* d_bytes, const int64_t* d_offsets, int64_t n,
                          const fd_ingest_out* d_out);
/* host pointers (staged through the device); synchronous */
int fd_ingest_json_host(fd_engine* eng, const uint8_t* bytes, const int64_t* offsets, int64_t n,
                        const fd_ingest_out* out);
/* the codec's scalar conversions on the host (diagnostics / tests): kind 0 = JSON number text -> f64
   (correctly rounded), 1 = amount text -> cents, 2 = ISO-8601 text -> epoch ms. flags: bit 0 grammar error,
   bit 1 inexact. */
int fd_ingest_scalar_host(int32_t kind, const uint8_t* text, int32_t n, double* f64_out, int64_t* i64_out,
                          int32_t* flags_out);

/* ---------------------------------------------------------------- diagnostics */
/* Per-launch device timing of the engine's hot kernels, measured with HIP events recorded on the
   launch stream around each kernel. fd_timing_read synchronises and returns the summed time (ms) and
   count of the timed launches of `kind` (FD_TIMING_ALL: every kind) since the last fd_timing_reset. */
enum fd_timing_kind { FD_TIMING_ALL = -1, FD_TIMING_XGB = 0, FD_TIMING_IFOREST = 1, FD_TIMING_FEATURES = 2,
                      FD_TIMING_BLEND = 3, FD_TIMING_ROUTE = 4, FD_TIMING_LSTM = 5,
                      FD_TIMING_WINDOWS = 6, FD_TIMING_INGEST = 7,
                      FD_TIMING_ENSEMBLE = 8 /* fused XGBoost + IsolationForest + blend kernel */ };
int fd_engine_set_timing(fd_engine* eng, int enable);
/* Engine tuning knobs (for A/B measurement; defaults are the tuned choices):
     "forest_kernel": 0 auto, 1 force the 256-thread kernel, 2 force the 1024-thread tree-split kernel
     on the threshold layout, 3 force the 1024-thread kernel on the binned layout, 6 force the tree-split
     small-batch path (auto takes it below 128 tiles of 256 transactions), 8 force the binned node-only-chunk
     kernel (auto's choice when the forest has that layout); the variants measured slower were removed
     "ensemble": 1 fused XGBoost + IsolationForest + blend kernel when applicable (default), 0 per-model kernels
     "ensemble_chunks": the fused kernel's chunk layout, 0 (default) auto: compact once the engine has RCCL
     communicators (fd_comm_init), else wide; 1 wide (24 XGBoost / 16 IsolationForest trees per chunk, 148 KB of
     LDS); 2 compact (20 / 12, 132 KB: room for an RCCL kernel on the same CU). Outputs are identical.
     "lstm_rows": LSTM tile, 0 auto (4 transactions below 4096, else 16), 4 or 16
     "timing_every": N >= 1, fd_engine_set_timing records HIP events on one launch in N of each timing kind
     (the others run without event records; fd_timing_read's launch count is the timed ones)
     "small_streams": latency batches (< 32768 transactions) with the LSTM head and / or several forests: 0
     (default) all on the engine stream (no cross-queue hops; config 5 0.088 ms per 1 k step), 1 the LSTM and the
     forests after the first on one side stream (0.095), 2 on two side streams (0.095)
     "pipeline_lean": fd_score_batch_pipelined's bucket pass, 1 (default) the lean kernel that fits beside the
     fused ensemble kernel, 0 the full bucket kernel
     "pipeline_gather": fd_score_batch_pipelined's batches of <= 4096 transactions (option slot_gather on, no slot
     stream), 1 (default) the gather bucket kernel (card slots found inside it: one feature launch), 0 the slot +
     lean bucket pair of the large batches
     (The compact rows' eight small-integer slots are always binned by one lookup in a per-plan table of the bins of
     0..31; round 5's option to search them instead was removed after its A/B)
     "ensemble_bin_global": the fused kernel's compact rows, 1 every varying slot binned by a search of its merged
     threshold table in global memory (L2-resident; no staging pass, chunk 0's DMA issued at the kernel's start),
     0 (default) the tables staged in LDS first (outputs identical)
     "lean_group": how the lean bucket kernel groups a bucket's keys by card (outputs identical): 2 (default) an
     LDS hash table of card slots (no sort), 1 a rank sort split over all threads, 0 the first m threads each rank
     one key over the whole list
     "latency_prebin": latency batches scored by the XGBoost + IsolationForest pair path with the LSTM head: the
     pair's tree-split binning in the LSTM launch (no binning launch; counter "latency_prebinned_batches"), 3
     (default) inside the LSTM's own workgroups, a binary-search level per recurrence step (2 where a thread would
     take more than two searches), 2 in extra workgroups after the LSTM's own, 1 ahead of them; 0 its own binning
     launch (outputs identical)
     (further options — "slot_stream", "slot_gather", "bucket_spread", "feature_prio", "ensemble_prio",
     "compact_vectors", "latency_fused", "seq_ring_lstm", "bucket_keys" — are listed with their measurements in
     DESIGN.md §3)
     "comm_timeout_ms": fd_sharded_step's split-size wait fails with FD_ERR_HIP after this many ms (default
     120000): a peer that never posts its counts (a dead rank, a different call pattern) becomes an error, not a hang
     "count_exchange": fd_sharded_step's per-peer counts as 1 one ncclAllGather per batch, 0 2 x world
     ncclSend/ncclRecv in the records group, -1 (default) the all-gather from 4 ranks (every rank the same; not while
     a prefetched batch is pending)
     "stream_priority": HIP priorities of the engine's pipeline and forward streams (ROCm keeps a hardware-queue
     pool per priority, so they stop sharing queues with the engine stream and RCCL's streams): 0 all default, 1
     the two pipeline streams high, 2 + the forward stream low, 3 (default) + the forward stream high. Set before
     the first pipelined call and fd_comm_init. */
int fd_engine_set_option(fd_engine* eng, const char* key, int64_t value);
/* Engine counters (diagnostics): "window_saturated" (sliding windows: transactions so far whose 24 h window held the
   ring's whole capacity K of prior events — their counts may be truncated at K; synchronises the engine's streams),
   "pipelined_batches" (batches through fd_score_batch_pipelined /
   fd_score_records_pipelined so far), "pipelined_compact_batches" (of those, scored by the fused ensemble kernel from
   the compact 64-B rows: no vectors requested), "pipelined_slot_stream_batches" (of those, with the slot pass on
   its own stream), "pipelined_host_ns" (host nanoseconds inside fd_score_batch_pipelined), "sharded_steps" (fd_sharded_step calls), "rccl_ops" (RCCL operations the exchanges issued: sends, receives,
   all-gathers) and "sharded_host_ns_<phase>" (host
   nanoseconds inside fd_sharded_step by phase: "wait" the split sizes, "partition" / "counts" / "count_copy" the
   next batch's route kernels, count exchange and copy to the host, "records" the records exchange, "score" the
   owner's pipeline launches, "back" / "scatter" the results exchange and the scatter into arrival order). */
int fd_engine_get_counter(fd_engine* eng, const char* key, int64_t* value);
int fd_timing_read(fd_engine* eng, int kind, double* total_ms, int64_t* launches);
int fd_timing_reset(fd_engine* eng);

#ifdef __cplusplus
}
#endif
#endif /* FDENGINE_H */
