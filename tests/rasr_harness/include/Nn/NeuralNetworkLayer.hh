// TEST DOUBLE: Nn::NeuralNetworkLayer<T> -- the accessors the GPU nn adapter's network unit reads
// (integration/rasr/Nn/GpuBatchFeatureScorerNetwork.cc), with the reference's "layer-type" names
// (src/Nn/NeuralNetworkLayer.cc:30-61) and dimension parameters (:68-76).  Parameters come from a "parameter-file"
// in a format of THIS double (little-endian f32: bias[out], then weights [in][out]), not RASR's file formats.
#pragma once
#include <cstdio>
#include <memory>
#include <cstdlib>
#include <string>
#include <vector>
#include <Core/Component.hh>
#include <Core/Types.hh>
namespace Nn {

template <class T>
class Matrix {  // weights_.at(input, output), column = output unit (LinearLayer.cc:405-419)
public:
    Matrix(u32 rows, u32 cols) : r_(rows), c_(cols), v_(static_cast<size_t>(rows) * cols) {}
    u32      nRows() const { return r_; }
    u32      nColumns() const { return c_; }
    T&       at(u32 i, u32 j) { return v_[static_cast<size_t>(j) * r_ + i]; }  // column-major, as RASR's
    const T& at(u32 i, u32 j) const { return v_[static_cast<size_t>(j) * r_ + i]; }

private:
    u32            r_, c_;
    std::vector<T> v_;
};

template <class T>
class Vector : public std::vector<T> {
public:
    explicit Vector(u32 n = 0) : std::vector<T>(n) {}
    T&       at(u32 i) { return (*this)[i]; }
    const T& at(u32 i) const { return (*this)[i]; }
};

template <class T>
class NeuralNetworkLayer : public Core::Component {
public:
    enum LayerType {
        identityLayer, sigmoidLayer, softmaxLayer, tanhLayer, rectifiedLayer, eluLayer, linearLayer,
        linearAndSigmoidLayer, linearAndSoftmaxLayer, linearAndTanhLayer, linearAndRectifiedLayer, linearAndEluLayer,
        unsupportedLayer
    };
    typedef Matrix<T> NnMatrix;
    typedef Vector<T> NnVector;

    NeuralNetworkLayer(const Core::Configuration& c, LayerType t, u32 in, u32 out)
            : Core::Component(c), type_(t), in_(in), out_(out) {}
    virtual ~NeuralNetworkLayer() {}
    static LayerType typeOf(const std::string& n) {
        static const char* const names[] = {"identity", "sigmoid", "softmax", "tanh", "rectified", "elu", "linear",
                                            "linear+sigmoid", "linear+softmax", "linear+tanh", "linear+rectified",
                                            "linear+elu"};
        for (int i = 0; i <= linearAndEluLayer; ++i)
            if (n == names[i])
                return static_cast<LayerType>(i);
        return unsupportedLayer;
    }
    static bool hasLinearPart(LayerType t) { return t >= linearLayer && t != unsupportedLayer; }

    LayerType getLayerType() const { return type_; }
    u32       nInputActivations() const { return 1; }
    u32       getInputActivationIndex(u32) const { return inputIndex_; }
    u32       getOutputActivationIndex() const { return outputIndex_; }
    u32       getInputDimension(u32) const { return in_; }
    u32       getOutputDimension() const { return out_; }
    NnMatrix* getWeights(u32) { return W_.get(); }
    NnVector* getBias() { return b_.get(); }

    // the network double wires the chain and loads the parameters
    void setActivationIndices(u32 in, u32 out) { inputIndex_ = in, outputIndex_ = out; }
    bool loadParameters(const std::string& file) {
        W_.reset(new NnMatrix(in_, out_));
        b_.reset(new NnVector(out_));
        FILE* f = std::fopen(file.c_str(), "rb");
        if (!f)
            return false;
        bool ok = std::fread(b_->data(), sizeof(T), out_, f) == out_;
        std::vector<T> w(static_cast<size_t>(in_) * out_);
        ok = ok && std::fread(w.data(), sizeof(T), w.size(), f) == w.size();
        std::fclose(f);
        for (u32 i = 0; ok && i < in_; ++i)
            for (u32 o = 0; o < out_; ++o)
                W_->at(i, o) = w[static_cast<size_t>(i) * out_ + o];
        return ok;
    }

private:
    LayerType                 type_;
    u32                       in_, out_, inputIndex_ = 0, outputIndex_ = 0;
    std::unique_ptr<NnMatrix> W_;
    std::unique_ptr<NnVector> b_;
};

}  // namespace Nn
