// TEST DOUBLE: Nn::NeuralNetwork<T> -- a chain of layers built from the configuration the way the reference names
// it (src/Nn/NeuralNetwork.cc:85-140): "neural-network.links = 0->layer-0:0" from the feature stream, each layer's
// "links" to the next one, per layer "layer-type", "dimension-input", "dimension-output", "parameter-file" (format of
// NeuralNetworkLayer.hh's double) and "gamma".  Only single chains (what the GPU adapter accepts); the output
// activation of layer l is l + 1 (one feature stream, NeuralNetwork.cc:140-142).
#pragma once
#include <memory>
#include <string>
#include <vector>
#include <Core/Assertions.hh>
#include <Core/Component.hh>
#include "LinearAndActivationLayer.hh"
#include "NeuralNetworkLayer.hh"
namespace Nn {
template <class T>
class NeuralNetwork : public Core::Component {
public:
    explicit NeuralNetwork(const Core::Configuration& c) : Core::Component(c) {}
    void initializeNetwork(u32 batchSize) {
        (void)batchSize;
        std::string link;
        if (!Configuration(config, "neural-network").get("links", link))
            criticalError("no configuration of neural network topology found");
        u32 in = 0;
        while (!link.empty()) {
            // "<source port>-><layer name>:<target port>"
            const size_t a = link.find("->"), b = link.rfind(':');
            verify(a != std::string::npos && b != std::string::npos && b > a);
            const std::string         name = link.substr(a + 2, b - a - 2);
            const Core::Configuration lc(config, name);
            std::string               type, v;
            verify(lc.get("layer-type", type));
            const u32 dimIn  = lc.get("dimension-input", v) ? static_cast<u32>(std::atoi(v.c_str())) : in;
            const u32 dimOut = lc.get("dimension-output", v) ? static_cast<u32>(std::atoi(v.c_str())) : dimIn;
            typedef NeuralNetworkLayer<T> L;
            const typename L::LayerType t = L::typeOf(type);
            L* layer = t == L::linearAndSoftmaxLayer ? new LinearAndSoftmaxLayer<T>(lc, dimIn, dimOut)
                                                     : new L(lc, t, dimIn, dimOut);
            layers_.emplace_back(layer);
            layer->setActivationIndices(static_cast<u32>(layers_.size() - 1), static_cast<u32>(layers_.size()));
            if (L::hasLinearPart(t)) {
                std::string file;
                if (!lc.get("parameter-file", file) || !layer->loadParameters(file))
                    criticalError("layer %s: cannot read its parameter file", name.c_str());
            }
            in = dimOut;
            if (!lc.get("links", link))
                link.clear();
        }
        if (layers_.empty())
            criticalError("empty network");
    }
    u32                     nLayers() const { return static_cast<u32>(layers_.size()); }
    NeuralNetworkLayer<T>&  getLayer(u32 l) { return *layers_.at(l); }
    NeuralNetworkLayer<T>&  getTopLayer() { return *layers_.back(); }
    void                    finishComputation() {}
    void                    initComputation() {}

private:
    typedef Core::Configuration Configuration;
    std::vector<std::unique_ptr<NeuralNetworkLayer<T>>> layers_;
};
}  // namespace Nn
