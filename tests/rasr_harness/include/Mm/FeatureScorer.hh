// TEST DOUBLE: the Mm::FeatureScorer plugin interface and its buffered protocol (method set and defaults as the
// interface the adapter is syntax-checked against)
#pragma once
#include <Core/Assertions.hh>
#include <Core/Component.hh>
#include <Core/ReferenceCounting.hh>
#include "Feature.hh"
#include "Types.hh"
namespace Mm {
class FeatureScorer : public virtual Core::Component, public Core::ReferenceCounted {
protected:
    class ContextScorer : public Core::ReferenceCounted {
    protected:
        ContextScorer() {}

    public:
        virtual ~ContextScorer() {}
        virtual EmissionIndex nEmissions() const           = 0;
        virtual Score         score(EmissionIndex e) const = 0;
    };

public:
    explicit FeatureScorer(const Core::Configuration& c) : Core::Component(c) {}
    virtual ~FeatureScorer() {}
    virtual EmissionIndex nMixtures() const                                            = 0;
    virtual void          getFeatureDescription(FeatureDescription& description) const = 0;

    typedef Core::Ref<const ContextScorer> Scorer;
    virtual Scorer getScorer(Core::Ref<const Feature>) const = 0;
    virtual Scorer getScorer(const FeatureVector&) const     = 0;
    virtual void   reset() const {}
    virtual void   finalize() const {}
    virtual bool   isBuffered() const { return false; }
    virtual void   addFeature(const FeatureVector&) const {}
    virtual void   addFeature(Core::Ref<const Feature>) const {}
    virtual Scorer flush() const { return Scorer(); }
    virtual bool   bufferFilled() const { return true; }
    virtual bool   bufferEmpty() const { return true; }
    virtual u32    bufferSize() const { return 0; }
};
}  // namespace Mm
