// TEST DOUBLE: Nn::LinearAndSoftmaxLayer<T> -- the top layer type the scorer requires, and removeLogPriorFromBias
// (src/Nn/LinearAndActivationLayer.hh:235-250: bias(c) -= prioriScale * prior(c) in T, nothing when the scale is 0)
#pragma once
#include <Core/Assertions.hh>
#include "NeuralNetworkLayer.hh"
#include "Prior.hh"
namespace Nn {
template <class T>
class LinearAndSoftmaxLayer : public NeuralNetworkLayer<T> {
public:
    LinearAndSoftmaxLayer(const Core::Configuration& c, u32 in, u32 out)
            : NeuralNetworkLayer<T>(c, NeuralNetworkLayer<T>::linearAndSoftmaxLayer, in, out) {}
    template <class S>
    void removeLogPriorFromBias(const Prior<S>& priors) {
        require(this->getBias());
        require_eq(priors.size(), this->getBias()->size());
        const T prioriScale = priors.scale();
        if (prioriScale != S(0.0))
            for (u32 c = 0; c < this->getBias()->size(); c++)
                this->getBias()->at(c) -= prioriScale * priors.at(c);
    }
};
}  // namespace Nn
