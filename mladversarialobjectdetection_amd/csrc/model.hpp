// model.hpp — EfficientDet victim description and the static op program executed by the HIP
// kernels.  The program is a topologically ordered op list over NHWC float32 tensors; its
// backward is the reversed list (data-gradient only: weights are constants of the attack).
//
// Architecture rules follow the reference's vendored automl code:
//   backbone      automl/efficientdet/backbone/efficientnet_model.py:129-151 (round_filters/
//                 round_repeats), :224-417 (MBConvBlock), :507-528 (Stem), :711-780 (features)
//                 efficientnet_builder.py:31-46,163-168 ; efficientnet_lite_builder.py:28-79
//   BiFPN         automl/efficientdet/tf2/efficientdet_keras.py:42-324, 700-775 ;
//                 tf2/fpn_configs.py:24-72
//   heads         automl/efficientdet/tf2/efficientdet_keras.py:327-632
//   configs       automl/efficientdet/hparams_config.py:170-467
#pragma once
#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace phx {

enum Act { ACT_NONE = 0, ACT_SWISH = 1, ACT_RELU6 = 2 };

enum OpT {
  OP_STEM = 0,      // 3x3 s2 conv, Cin=3, no bias
  OP_PW = 1,        // 1x1 conv (+bias)
  OP_DW = 2,        // depthwise kxk conv, stride s, TF SAME, no bias
  OP_BN = 3,        // batch norm (+activation)
  OP_SE = 4,        // squeeze-excite: x * sigmoid(W2 act(W1 mean(x) + b1) + b2)
  OP_ADD = 5,       // residual add
  OP_MAXPOOL = 6,   // k x k max pool, stride s, TF SAME (-inf pad)
  OP_UPSAMPLE = 7,  // nearest neighbour (tf.compat.v1 resize_nearest_neighbor)
  OP_FUSE = 8,      // BiFPN node fuse (fastattn / sum) followed by activation
};

struct Tensor {
  int n = 0, h = 0, w = 0, c = 0;
  size_t off = 0;     // float offset in the activation arena
  long goff = -1;     // float offset in the gradient arena, -1 = no gradient
  int level = -1;     // pyramid level (heads), informative
  size_t numel() const { return (size_t)n * h * w * c; }
  size_t rows() const { return (size_t)n * h * w; }
};

struct Op {
  OpT t;
  int in[3] = {-1, -1, -1};
  int nin = 0;
  int out = -1;
  int k = 1, stride = 1, pad_t = 0, pad_l = 0, act = ACT_NONE;
  long w = -1, wt = -1, b = -1;                    // weights (float offsets), wt = transposed
  long gamma = -1, beta = -1, mmean = -1, mvar = -1;
  int slot = -1;                                   // BN / SE statistics slot
  long w1 = -1, b1 = -1, w2 = -1, b2 = -1;         // SE
  int cse = 0;
  long wsm[3] = {-1, -1, -1};
  int fuse_method = 0;                             // 0 fastattn, 1 sum
  bool acc[3] = {false, false, false};             // backward: accumulate into input grad
  bool bwd = false;                                // op participates in the backward pass
  float survival = 0.f;                            // OP_ADD: drop connect on in[0] (0 = off)
  int drop_block = -1;                             // its MBConv block index (Philox counter)
  std::string name;
};

struct WeightEntry {
  std::string name;
  std::vector<int> shape;
  size_t offset;
  std::string kind;  // kernel, bias, gamma, beta, moving_mean, moving_variance, wsm
};

struct ModelConfig {
  std::string name;
  std::string backbone;
  int image_size = 512;
  int fpn_num_filters = 64;
  int fpn_cell_repeats = 3;
  int box_class_repeats = 3;
  int min_level = 3, max_level = 7;
  int num_classes = 90;
  int num_scales = 3;
  std::vector<float> aspect_ratios{1.0f, 2.0f, 0.5f};
  float anchor_scale = 4.0f;
  int act = ACT_SWISH;
  int fpn_weight_method = 0;  // 0 fastattn, 1 sum
  float mean_rgb[3] = {0.485f * 255, 0.456f * 255, 0.406f * 255};
  float stddev_rgb[3] = {0.229f * 255, 0.224f * 255, 0.225f * 255};
  // backbone
  double width_coefficient = 1.0, depth_coefficient = 1.0;
  bool lite = false;             // relu6, no SE, fixed stem/head
  double survival_prob = 0.0;    // drop connect (0 = off); b0 disables it
  int num_anchors() const { return num_scales * (int)aspect_ratios.size(); }
};

// Fills `cfg` for one of the reference's model names; returns false if unknown.
bool get_model_config(const std::string& model_name, ModelConfig* cfg);

struct Program {
  std::vector<Tensor> tensors;
  std::vector<Op> ops;
  int input = -1;
  std::vector<int> cls_out, box_out;   // per level
  size_t act_floats = 0, grad_floats = 0;
  int n_slots = 0;                     // BN + SE statistics slots
  std::vector<int> slot_channels;      // channels per slot
  int batch = 0;
};

// Walks the victim architecture.  With batch == 0 only the weight manifest is produced.
class NetBuilder {
 public:
  // training: drop-connect active (attack step, training=True); ignored when batch == 0
  NetBuilder(const ModelConfig& cfg, int batch, bool training = true);
  void build();
  const std::vector<WeightEntry>& weights() const { return weights_; }
  size_t weight_floats() const { return wfloats_; }
  Program& program() { return prog_; }

 private:
  int new_tensor(int n, int h, int w, int c);
  long wref(const std::string& name, std::vector<int> shape, const std::string& kind);
  int op_stem(int x, const std::string& pfx, int cout);
  int op_pw(int x, const std::string& wname, int cout, bool bias);
  int op_dw(int x, const std::string& wname, int k, int stride);
  int op_bn(int x, const std::string& pfx, int act);
  int op_se(int x, const std::string& pfx, int cse);
  int op_add(int a, int b);
  int op_maxpool(int x, int k, int stride, int oh, int ow);
  int op_upsample(int x, int oh, int ow);
  int op_fuse(const std::vector<int>& xs, const std::string& pfx, int act);
  int sepconv(int x, const std::string& pfx, int cout);

  void build_backbone(std::vector<int>* feats);
  int resample(int x, int target_h, int target_w, const std::string& pfx);
  void plan_backward();

  ModelConfig cfg_;
  int batch_;
  bool training_;
  Program prog_;
  std::vector<WeightEntry> weights_;
  std::map<std::string, long> wmap_;
  size_t wfloats_ = 0;
};

}  // namespace phx
