"""mep_amd: MI355X-native tri-modal residual-attention training path."""
